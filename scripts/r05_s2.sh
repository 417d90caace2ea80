#!/bin/bash
# r05 session 2: where the SAH trees' outliers come from under the pair order (diff masks), and the A/B perf
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05s2; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u scripts/parity_report.py --configs C2d1,C2 --frames 0 --modes bench,sah_nogroup,exact_sah,lbvh \
  --save-diff $O/diff_new --out $O/parity_new.json > $O/parity_new.log 2>&1 || { echo "new rc=$?"; tail -5 $O/parity_new.log; exit 1; }
grep '^{"pixels' $O/parity_new.log | python3 -c "
import json,sys
for l in sys.stdin: d=json.loads(l); print('new', d['config'], d['mode'], d['outliers_gt1'], d['max_lsb'])"
RTAMD_LIB=$PWD/real-time-gpu-ray-tracer_amd/lib/librtamd_r04base.so timeout -k 10 400 python -u scripts/parity_report.py --configs C2d1,C2 --frames 0 \
  --modes bench,sah_nogroup,lbvh --save-diff $O/diff_old --out $O/parity_old.json > $O/parity_old.log 2>&1 || { echo "old rc=$?"; tail -5 $O/parity_old.log; exit 1; }
grep '^{"pixels' $O/parity_old.log | python3 -c "
import json,sys
for l in sys.stdin: d=json.loads(l); print('old', d['config'], d['mode'], d['outliers_gt1'], d['max_lsb'])"
OPT=lib VALS="default r04base" REPS=2 CASES="c2|--steps 100;c3|--config C3 --steps 40;c5|--config C5 --build lbvh --steps 12 --warmup 3;c5rb|--config C5 --build lbvh --rebuild --steps 12 --warmup 3" bash scripts/ab.sh r05s2_ab
