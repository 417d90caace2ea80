#!/bin/bash
# r05 session 19: option "split_cus" (CU-masked scene stream for the per-frame BLAS rebuild, lanes on the rest), C5
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05s19; mkdir -p $O
export TMPDIR=/tmp
one() {   # name args...
  local name=$1; shift 1
  timeout -k 10 300 python3 bench.py "$@" --no-cpu-baseline > $O/$name.log 2>&1 || { echo "fail $name"; tail -5 $O/$name.log; exit 1; }
  python3 - $O/$name.log $name <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().split("\n")[-1])
print(f"{sys.argv[2]:18s} lanes {d['config']['overlap_lanes']} ms/frame {d['ms_per_step']:.4f} lat {d['frame_latency_ms_median']:.4f} serial {d['kernel_ms']:.4f}", flush=True)
PY
}
for rep in 1 2; do
  for p in 0 10 15 20 25 30; do
    one c5rb_split${p}_$rep --config C5 --build lbvh --rebuild --steps 12 --warmup 3 --pre-opt split_cus=$p
  done
done
one c5rb_split20_L3 --config C5 --build lbvh --rebuild --steps 12 --warmup 3 --pre-opt split_cus=20 --overlap 3
one c5_split0 --config C5 --build lbvh --steps 12 --warmup 3
one c5_split20 --config C5 --build lbvh --steps 12 --warmup 3 --pre-opt split_cus=20
