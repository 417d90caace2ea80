#!/bin/bash
# r05 session 4: visit order (pairs / entry t) x TLAS (median leaf 2 / median leaf 1 / SAH): parity + perf
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05s4; mkdir -p $O
export TMPDIR=/tmp
M="bench,bench+tlas_median_leaf=1,bench+wide_order=0,bench+wide_order=0+tlas_median_leaf=1,bench+wide_order=0+tlas_sah=1"
timeout -k 10 500 python -u scripts/parity_report.py --configs C2d1,C2,C3 --frames 0,37 --modes $M \
  --out $O/parity.json > $O/parity.log 2>&1 || { echo "rc=$?"; tail -5 $O/parity.log; exit 1; }
grep '^{"pixels' $O/parity.log | python3 -c "
import json,sys
for l in sys.stdin: d=json.loads(l); print(d['config'], d['mode'], d['frame'], d['outliers_gt1'], d['max_lsb'])"
OPT=opts VALS="base tlas_median_leaf=1 wide_order=0 wide_order=0,tlas_median_leaf=1 wide_order=0,tlas_sah=1" REPS=2 \
  CASES="c2|--steps 100;c3|--config C3 --steps 40" bash scripts/ab.sh r05s4_ab
