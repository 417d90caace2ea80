#!/bin/bash
# Round 4 step 20: C5 rebuild with the scene stream at a higher HIP priority
set -o pipefail
O=gpurun_out/r04s20; mkdir -p $O
export TMPDIR=/tmp
python3 -c "
import ctypes; h=ctypes.CDLL('libamdhip64.so'); lo=ctypes.c_int(); hi=ctypes.c_int()
print('priority range', h.hipDeviceGetStreamPriorityRange(ctypes.byref(lo), ctypes.byref(hi)), lo.value, hi.value)"
i=0
for args in "--pre-opt scene_priority=-1" "--pre-opt scene_priority=-1 --overlap 3" "" "--pre-opt scene_priority=-1 --overlap 4"; do
  i=$((i+1))
  timeout -k 10 300 python -u bench.py --config C5 --build lbvh --rebuild --steps 12 --warmup 3 --no-cpu-baseline $args \
    > $O/c5_$i.log 2>&1 || { echo "rc=$? $args"; tail -3 $O/c5_$i.log; continue; }
  grep '^{' $O/c5_$i.log | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('c5 rebuild $args', d['ms_per_step'], d['config']['overlap_lanes'])"
done
