#!/bin/bash
# r05 session 1: reference pair order in quads — parity counts + A/B against the round-4 library
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05s1; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity_full.py -k "bench_configuration or reference_trees or reference_order" -v -s --timeout 300 --timeout-method thread > $O/parity.log 2>&1
echo "parity rc=$?"; grep -E "outliers|differ|passed|failed" $O/parity.log | tail -40
timeout -k 10 300 python -u -m pytest tests/test_gpu_lbvh.py -k "quad_collapse" -q --timeout 200 --timeout-method thread > $O/lbvh.log 2>&1 || { echo "lbvh test failed"; tail -20 $O/lbvh.log; exit 1; }
tail -1 $O/lbvh.log
OPT=lib VALS="default r04base" REPS=2 CASES="c2|--steps 100;c3|--config C3 --steps 40;c5|--config C5 --build lbvh --steps 12 --warmup 3;c5rb|--config C5 --build lbvh --rebuild --steps 12 --warmup 3" scripts/ab.sh r05s1_ab
