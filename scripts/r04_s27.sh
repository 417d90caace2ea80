#!/bin/bash
# Round 4 step 27: C5 rebuild (2 lanes off the null stream): slots left to the rebuild, interleaved with the default
set -o pipefail
O=gpurun_out/r04s27; mkdir -p $O
export TMPDIR=/tmp
i=0
for args in "" "--opt reserve=256" "--opt grid_pct=85" "" "--opt reserve=128" "--opt grid_pct=67" ""; do
  i=$((i+1))
  timeout -k 10 300 python -u bench.py --config C5 --build lbvh --rebuild --steps 12 --warmup 3 --no-cpu-baseline $args \
    > $O/c5_$i.log 2>&1 || exit 1
  grep '^{' $O/c5_$i.log | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('c5 rebuild $args', d['ms_per_step'])"
done
