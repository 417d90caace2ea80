#!/bin/bash
# r05 session 3: the reference's median TLAS under SAH BLASes (pair order everywhere): parity + perf
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05s3; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u scripts/parity_report.py --configs C2d1,C2,C3 --frames 0,37 --modes bench,bench+tlas_sah=1 \
  --out $O/parity.json > $O/parity.log 2>&1 || { echo "rc=$?"; tail -5 $O/parity.log; exit 1; }
grep '^{"pixels' $O/parity.log | python3 -c "
import json,sys
for l in sys.stdin: d=json.loads(l); print(d['config'], d['mode'], d['frame'], d['outliers_gt1'], d['max_lsb'])"
OPT=tlas_sah VALS="0 1" REPS=2 CASES="c2|--steps 100;c3|--config C3 --steps 40;c4s|--config C4 --steps 100 --shard 0/8" bash scripts/ab.sh r05s3_ab
