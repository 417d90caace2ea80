#!/bin/bash
# r05 session 34: C2 1/8 share, final library (default path and a copy via RTAMD_LIB) vs the previous final library b8c1a1be
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05s34; mkdir -p $O
export TMPDIR=/tmp
L=$PWD/real-time-gpu-ray-tracer_amd/lib
for rep in 1 2 3; do
  for v in prev cur default; do
    lib=""; [ $v != default ] && lib=$L/librtamd_$v.so
    RTAMD_LIB=$lib timeout -k 10 300 python3 bench.py --steps 100 --shard 0/8 --no-cpu-baseline > $O/share_${v}_$rep.log 2>&1 || { echo fail; tail -3 $O/share_${v}_$rep.log; exit 1; }
    python3 -c "
import json
d=json.loads(open('$O/share_${v}_$rep.log').read().strip().split('\n')[-1]); print('$v', d['ms_per_step'], d['config']['overlap_lanes'], d['frame_latency_ms_median'])"
  done
done
