#!/bin/bash
# r05 session 7: visit order per tree family (SAH: greedy quads by entry t; compat / LBVH: two-level quads in pair order)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05s7; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity_full.py -k "bench_configuration or reference_trees" -s -v --timeout 300 --timeout-method thread > $O/parity.log 2>&1
echo "parity rc=$?"; grep -E "outliers|differ|passed|failed" $O/parity.log | grep -v "^tests" | tail -40
timeout -k 10 300 python -u -m pytest tests/test_gpu_lbvh.py tests/test_gpu_group.py -q --timeout 200 --timeout-method thread > $O/lbvh.log 2>&1; echo "lbvh/group rc=$?"; tail -2 $O/lbvh.log
OPT=lib VALS="default r04base" REPS=2 CASES="c2|--steps 100;c3|--config C3 --steps 40;c5|--config C5 --build lbvh --steps 12 --warmup 3;c5rb|--config C5 --build lbvh --rebuild --steps 12 --warmup 3" bash scripts/ab.sh r05s7_ab
