#!/bin/bash
# r05 session 33: every rebuild frame on 2 library lanes: C2-LBVH and C5 whole frames, C5 share; plus the caller-lane
# "classic" form for C2-LBVH for comparison
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05s33; mkdir -p $O
export TMPDIR=/tmp
one() {   # name args...
  local name=$1; shift 1
  timeout -k 10 400 python3 bench.py "$@" --no-cpu-baseline > $O/$name.log 2>&1 || { echo "fail $name"; tail -5 $O/$name.log; exit 1; }
  python3 - $O/$name.log $name <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().split("\n")[-1])
print(f"{sys.argv[2]:18s} lanes {d['config']['overlap_lanes']} ms/frame {d['ms_per_step']:.4f} lat {d['frame_latency_ms_median']:.4f} serial {d['kernel_ms']:.4f}", flush=True)
PY
}
for rep in 1 2; do
  one c2lrb_lib_$rep --build lbvh --rebuild --steps 60
  one c2lrb_caller2_$rep --build lbvh --rebuild --steps 60 --lanes caller --overlap 2
  one c5rb_lib_$rep --config C5 --build lbvh --rebuild --steps 12 --warmup 3
  one c5rb_s0_$rep --config C5 --build lbvh --rebuild --steps 24 --warmup 4 --shard 0/8
  one c2l_$rep --build lbvh --steps 100
done
