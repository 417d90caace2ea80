#!/bin/bash
# r05 session 24: a synchronous call takes the whole grid (syncfull) and bench's last timed frame is that call;
# the driver's 20-step window and the 100-step line against HEAD's library (r05b) with the same bench.py
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05s24; mkdir -p $O
export TMPDIR=/tmp
L=$PWD/real-time-gpu-ray-tracer_amd/lib
one() {   # name lib args...
  local name=$1 v=$2; shift 2
  local lib=""; [ $v != default ] && lib=$L/librtamd_$v.so
  RTAMD_LIB=$lib timeout -k 10 300 python3 bench.py "$@" --no-cpu-baseline > $O/${name}_$v.log 2>&1 || { echo "fail $name $v"; tail -5 $O/${name}_$v.log; exit 1; }
  python3 - $O/${name}_$v.log $name $v <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().split("\n")[-1])
print(f"{sys.argv[2]:10s} {sys.argv[3]:9s} ms/frame {d['ms_per_step']:.4f} lat {d['frame_latency_ms_median']:.4f} serial {d['kernel_ms']:.4f}", flush=True)
PY
}
for rep in 1 2 3; do
  for v in syncfull r05b; do
    ba=""; [ $v = r05b ] && ba="--burst-end async"
    one drv_$rep $v --gpus 1 --steps 20 --warmup 5 $ba
    one c2_$rep $v --steps 100 $ba
    one c3_$rep $v --config C3 --steps 40 $ba
  done
  one drv_async_$rep syncfull --gpus 1 --steps 20 --warmup 5 --burst-end async
done
