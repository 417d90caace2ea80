#!/bin/bash
# r05 session 5: the hierarchical quad order without a sort network: parity + perf against round 4
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05s5; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u scripts/parity_report.py --configs C2d1,C2,C3 --frames 0,37 --modes bench,bench+tlas_median_leaf=1 \
  --out $O/parity.json > $O/parity.log 2>&1 || { echo "rc=$?"; tail -5 $O/parity.log; exit 1; }
grep '^{"pixels' $O/parity.log | python3 -c "
import json,sys
for l in sys.stdin: d=json.loads(l); print(d['config'], d['mode'], d['frame'], d['outliers_gt1'], d['max_lsb'])"
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity_full.py -k "bench_configuration and C5" -s -q --timeout 300 --timeout-method thread > $O/c5.log 2>&1
echo "c5 rc=$?"; grep -E "outliers|passed|failed" $O/c5.log
OPT=lib VALS="default r04base" REPS=2 CASES="c2|--steps 100;c3|--config C3 --steps 40;c5|--config C5 --build lbvh --steps 12 --warmup 3;c5rb|--config C5 --build lbvh --rebuild --steps 12 --warmup 3" bash scripts/ab.sh r05s5_ab
OPT=tlas_median_leaf VALS="0 1" REPS=2 CASES="c2|--steps 100;c3|--config C3 --steps 40" bash scripts/ab.sh r05s5_ab2
