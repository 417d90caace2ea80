#!/bin/bash
# Round 4 step 28: C5 rebuild on 2 lanes: hardware queues per process
set -o pipefail
O=gpurun_out/r04s28; mkdir -p $O
export TMPDIR=/tmp
i=0
for q in 12 4 8 12 4 24; do
  i=$((i+1))
  RTAMD_HWQ=$q timeout -k 10 300 python -u bench.py --config C5 --build lbvh --rebuild --steps 12 --warmup 3 --no-cpu-baseline \
    > $O/c5_$i.log 2>&1 || exit 1
  grep '^{' $O/c5_$i.log | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('c5 rebuild hwq=$q', d['ms_per_step'])"
done
