#!/bin/bash
# Round 4 step 19: kernel timeline of the C5 rebuild pipeline at the new defaults (2 lanes off the null stream)
set -o pipefail
O=gpurun_out/r04s19; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/kt -o run --output-format csv -- python -u bench.py --config C5 --build lbvh \
  --rebuild --steps 12 --warmup 3 --no-cpu-baseline > $O/kt.log 2>&1 || exit 1
grep '^{' $O/kt.log | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('c5 rebuild', d['ms_per_step'])"
