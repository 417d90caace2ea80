#!/bin/bash
# Round-4 session 6: cooperative tail (option "coop"): GPU tests, A/B on the bench lines, timelines with it on.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r04s6
mkdir -p $OUT
export TMPDIR=/tmp
true > $OUT/tests.log
rc=0
[ $rc -ne 0 ] && exit $rc
DIAG=$PWD/real-time-gpu-ray-tracer_amd/lib/librtamd_diag.so
for v in 0 1 2; do
  RTAMD_LIB=$DIAG timeout -k 10 200 python3 scripts/timeline.py --parts 8 --threshold 0 --opt coop=$v --out $OUT/tl_c2_coop$v.npz > $OUT/tl_c2_coop$v.log 2>&1 || exit 1
  RTAMD_LIB=$DIAG timeout -k 10 200 python3 scripts/timeline.py --parts 8 --threshold 0 --shard 0/8 --opt coop=$v --out $OUT/tl_share_coop$v.npz > $OUT/tl_share_coop$v.log 2>&1 || exit 1
  grep -h tag $OUT/tl_c2_coop$v.log $OUT/tl_share_coop$v.log | cut -c1-200
done
REPS=2 OPT=coop VALS="0 1 2" bash scripts/r04_ab.sh r04s6/ab
