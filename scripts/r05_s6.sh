#!/bin/bash
# r05 session 6: traversal work per ray, round-4 library against the pair-order library
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05s6; mkdir -p $O
export TMPDIR=/tmp
B=$PWD/real-time-gpu-ray-tracer_amd/lib/librtamd_r04base.so
run() { timeout -k 10 300 "$@" >> $O/work.jsonl 2>> $O/err.log || { echo "rc=$? $*"; tail -5 $O/err.log; exit 1; }; }
for c in C2 C3; do
  RTAMD_LIB=$B run python3 scripts/work_counts.py --config $c --tag r04
  run python3 scripts/work_counts.py --config $c --tag new
  run python3 scripts/work_counts.py --config $c --tag new_leaf1 --opt tlas_median_leaf=1
  run python3 scripts/work_counts.py --config $c --tag new_tlas_sah --opt tlas_sah=1
done
RTAMD_LIB=$B run python3 scripts/work_counts.py --config C5 --build lbvh --tag r04
run python3 scripts/work_counts.py --config C5 --build lbvh --tag new
cat $O/work.jsonl
