#!/bin/bash
# r05 session 20: C5 with the per-frame rebuild: persistent grid 75..100 % (room for the rebuild's kernels), 2 / 3 BLAS sets
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05s20; mkdir -p $O
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
  for g in 100 95 90 85 75; do
    one c5rb_g${g}_$rep --config C5 --build lbvh --rebuild --steps 12 --warmup 3 --opt grid_pct=$g
  done
  one c5rb_g90_s3_$rep --config C5 --build lbvh --rebuild --steps 12 --warmup 3 --opt grid_pct=90 --pre-opt blas_sets=3
done
