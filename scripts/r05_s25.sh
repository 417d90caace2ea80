#!/bin/bash
# r05 session 25: claim ahead (RT_CLAIM_AHEAD: a wave claims its band's next item when it consumes one, so the queue
# atomic's round trip overlaps the refill and traversal) against HEAD (r05b)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05s25; mkdir -p $O
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
for rep in 1 2 3; do
  for v in ahead r05b; do
    one c2_$rep $v --steps 100
    one c2ser_$rep $v --steps 40 --overlap 1
    one drv_$rep $v --gpus 1 --steps 20 --warmup 5
    one share8_$rep $v --steps 100 --shard 0/8
    one c3_$rep $v --config C3 --steps 40
  done
done
for v in ahead r05b; do
  one c5_1 $v --config C5 --build lbvh --steps 12 --warmup 3
  one c5ser_1 $v --config C5 --build lbvh --steps 6 --warmup 2 --overlap 1
done
