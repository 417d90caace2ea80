#!/bin/bash
# r05 session 47: waves whose queue is dry raise their issue priority (s_setprio 2: the launch's tail issues ahead of
# waves that still have queue work, and ahead of the next lane's launch) — diagnostic build of trace_kernel.hip
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05s47; mkdir -p $O
export TMPDIR=/tmp
L=$PWD/real-time-gpu-ray-tracer_amd/lib
one() {   # lib name args...
  local v=$1 name=$2; shift 2
  lib=""; [ $v != default ] && lib=$L/librtamd_$v.so
  RTAMD_LIB=$lib timeout -k 10 400 python3 bench.py "$@" --no-cpu-baseline > $O/$name.log 2>&1 || { echo "fail $name"; tail -5 $O/$name.log; exit 1; }
  python3 - $O/$name.log $name <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().split("\n")[-1])
print(f"{sys.argv[2]:18s} ms/frame {d['ms_per_step']:.4f} lat {d['frame_latency_ms_median']:.4f} serial {d['kernel_ms']:.4f}", flush=True)
PY
}
for rep in 1 2; do
  for v in default prio; do
    one $v c2_${v}_$rep --steps 100
    one $v drv_${v}_$rep --steps 20 --warmup 5
    one $v c3_${v}_$rep --config C3 --steps 40
    one $v c5_${v}_$rep --config C5 --build lbvh --steps 12 --warmup 3
  done
done
