#!/bin/bash
# r05 session 8: box decisions inside the error margin re-taken with the reference's slab — residual + cost
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05s8; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity_full.py -k "bench_configuration or reference_trees" -s -v --timeout 300 --timeout-method thread > $O/parity.log 2>&1
echo "parity rc=$?"; grep -E "outliers of|differ" $O/parity.log | sed 's/^tests.*\] //' | tail -40
OPT=lib VALS="default r05a" REPS=2 CASES="c2|--steps 100;c3|--config C3 --steps 40;c5|--config C5 --build lbvh --steps 12 --warmup 3;c2s|--steps 100 --overlap 1" bash scripts/ab.sh r05s8_ab
timeout -k 10 600 python -u -m pytest tests/test_gpu_fake_rccl.py tests/test_gpu_edges.py tests/test_gpu_lbvh.py -v --timeout 300 --timeout-method thread > $O/fake_rccl.log 2>&1
echo "fake_rccl/edges rc=$?"; grep -E "PASS|FAIL|passed|failed|world" $O/fake_rccl.log | tail -20
