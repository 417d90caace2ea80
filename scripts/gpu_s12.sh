#!/bin/bash
# Round-6 session: 16 library lanes — the lane tests, then C2 / C4 1/8 shares and the whole C2 frame at 6-16 lanes.
cd ${GRAFT_REPO_ROOT:-$(dirname "$0")/..}
export TMPDIR=/tmp
OUT=gpurun_out/${S_OUT:-r06s12}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_edges.py tests/test_gpu_fake_rccl.py tests/test_gpu_multigpu.py -q -rf --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $OUT/tests.log; [ $rc -ne 0 ] && exit $rc
OPT=overlap VALS="8 12 16" REPS=2 CASES="c2s8|--steps 100 --shard 0/8;c4s8|--config C4 --steps 100 --shard 2/8" bash scripts/ab.sh ${S_OUT:-r06s12}/shares || exit 1
OPT=overlap VALS="4 6 8" REPS=2 CASES="c2_20|--steps 20 --warmup 5;c2_100|--steps 100" bash scripts/ab.sh ${S_OUT:-r06s12}/whole
