#!/bin/bash
# Round 4 step 14: C5 rebuild beside the trace: reserved persistent slots for the rebuild kernels
set -o pipefail
O=gpurun_out/r04s14; mkdir -p $O
export TMPDIR=/tmp
for args in "--rebuild --opt reserve=64" "--rebuild --opt reserve=128" "--rebuild --opt reserve=256" "--rebuild" "--opt reserve=128"; do
  tag=$(echo "x$args" | tr -d ' -' | tr '=' '_')
  timeout -k 10 300 python -u bench.py --config C5 --build lbvh --steps 12 --warmup 3 --no-cpu-baseline $args \
    > $O/c5_$tag.log 2>&1 || exit 1
  grep '^{' $O/c5_$tag.log | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('c5 $tag', d['ms_per_step'], d['kernel_ms'])"
done
