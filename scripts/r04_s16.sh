#!/bin/bash
# Round 4 step 16: C5 rebuild: hardware queues / lane streams (the scene stream shared a queue with lane 0)
set -o pipefail
O=gpurun_out/r04s16; mkdir -p $O
export TMPDIR=/tmp
i=0
for spec in "12|--lane-priority 0" "12|" "8|--lane-priority 0" "4|--lane-priority 0" "4|"; do
  i=$((i+1)); q=${spec%%|*}; args=${spec#*|}
  RTAMD_HWQ=$q timeout -k 10 300 python -u bench.py --config C5 --build lbvh --rebuild --steps 12 --warmup 3 --no-cpu-baseline $args \
    > $O/c5_$i.log 2>&1 || exit 1
  grep '^{' $O/c5_$i.log | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('c5 rebuild hwq=$q $args', d['ms_per_step'])"
done
