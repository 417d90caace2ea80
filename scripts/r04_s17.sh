#!/bin/bash
# Round 4 step 17: C5 rebuild on lanes off the null stream: lane count, reserved slots
set -o pipefail
O=gpurun_out/r04s17; mkdir -p $O
export TMPDIR=/tmp
i=0
for args in "" "--overlap 3" "--overlap 3 --opt reserve=64" "--overlap 4 --opt reserve=64" "--overlap 2"; do
  i=$((i+1))
  timeout -k 10 300 python -u bench.py --config C5 --build lbvh --rebuild --steps 12 --warmup 3 --no-cpu-baseline $args \
    > $O/c5_$i.log 2>&1 || exit 1
  grep '^{' $O/c5_$i.log | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('c5 rebuild $args', d['ms_per_step'], d['config']['overlap_lanes'])"
done
