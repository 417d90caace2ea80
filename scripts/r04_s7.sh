#!/bin/bash
# Round-4 session 7: C5 full-frame parity by tree / group / visit order; joiners (alone-only rule) A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r04s7
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python3 -u scripts/parity_report.py --configs C5 --frames 0 \
    --modes lbvh,lbvh_nogroup,fast_compat,fast_compat_binary --out $OUT/parity_c5.json > $OUT/parity_c5.log 2>&1
rc=$?; echo "parity rc=$rc"; grep -h '"mode"' $OUT/parity_c5.log | cut -c1-220
[ $rc -ne 0 ] && { tail -20 $OUT/parity_c5.log; exit $rc; }
CASES="c2_20|--steps 20 --warmup 5;c2_100|--steps 100;share8|--steps 100 --shard 0/8;c3|--config C3 --steps 40" \
  REPS=2 OPT=joiners VALS="0 1" bash scripts/r04_ab.sh r04s7/ab
