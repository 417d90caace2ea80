#!/bin/bash
# r05 session 23: BLAS-leaf deferral (RT_LEAF_DEFER K: a round's BLAS leaves wait when fewer than K lanes hold one
# beside instance entries) against the same source with K = 0 (defer0) and HEAD (r05b)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05s23; mkdir -p $O
export TMPDIR=/tmp
L=$PWD/real-time-gpu-ray-tracer_amd/lib
one() {   # name lib args...
  local name=$1 v=$2; shift 2
  local lib=""; [ $v != default ] && lib=$L/librtamd_$v.so
  RTAMD_LIB=$lib timeout -k 10 300 python3 bench.py "$@" --no-cpu-baseline > $O/${name}_$v.log 2>&1 || { echo "fail $name $v"; tail -5 $O/${name}_$v.log; exit 1; }
  python3 - $O/${name}_$v.log $name $v <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().split("\n")[-1])
print(f"{sys.argv[2]:10s} {sys.argv[3]:8s} ms/frame {d['ms_per_step']:.4f} lat {d['frame_latency_ms_median']:.4f} serial {d['kernel_ms']:.4f}", flush=True)
PY
}
for rep in 1 2; do
  for v in defer0 defer4 defer8 defer16 r05b; do
    one c3_$rep $v --config C3 --steps 40
    one c3ser_$rep $v --config C3 --steps 20 --overlap 1
    one c5_$rep $v --config C5 --build lbvh --steps 12 --warmup 3
    one c2_$rep $v --steps 100
  done
done
