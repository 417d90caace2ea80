#!/bin/bash
# Round 4 step 9: the C5 rebuild alone (time + kernel breakdown), and C5 rebuild pipelines
set -o pipefail
O=gpurun_out/r04s9; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/rebuild_alone.py --config C5 > $O/alone.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kst_alone -o run --output-format csv -- python -u scripts/rebuild_alone.py \
  --config C5 > $O/kst_alone.log 2>&1 || exit 1
for args in "--overlap 3" "--overlap 2" "--overlap 4" "--overlap 3 --opt grid_pct=100" "--overlap 3 --opt grid_pct=75"; do
  tag=$(echo "$args" | tr -d ' -' | tr '=' '_')
  timeout -k 10 300 python -u bench.py --config C5 --build lbvh --rebuild --steps 12 --warmup 3 --no-cpu-baseline $args \
    > $O/b_$tag.log 2>&1 || exit 1
  grep '^{' $O/b_$tag.log | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('$tag', d['ms_per_step'])"
done
