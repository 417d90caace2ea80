#!/bin/bash
# Round 4 step 18: C5 lanes (with and without the rebuild)
set -o pipefail
O=gpurun_out/r04s18; mkdir -p $O
export TMPDIR=/tmp
i=0
for args in "--rebuild --overlap 1" "--rebuild --overlap 2" "--rebuild --overlap 2 --opt blas_sets=2" "--rebuild --overlap 2 --opt grid_pct=75" "--overlap 2" "--overlap 3" ""; do
  i=$((i+1))
  timeout -k 10 300 python -u bench.py --config C5 --build lbvh --steps 12 --warmup 3 --no-cpu-baseline $args \
    > $O/c5_$i.log 2>&1 || exit 1
  grep '^{' $O/c5_$i.log | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('c5 $args', d['ms_per_step'], d['config']['overlap_lanes'])"
done
