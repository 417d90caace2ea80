#!/bin/bash
# r05 session 27: option "tlas_after_build" (a rebuilding frame's records / TLAS on the scene stream right behind the
# BLAS rebuild) on C5 and C2 with the per-frame rebuild
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05s27; mkdir -p $O
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
for rep in 1 2 3; do
  for t in 0 1; do
    one c5rb_t${t}_$rep --config C5 --build lbvh --rebuild --steps 12 --warmup 3 --opt tlas_after_build=$t
    one c2rb_t${t}_$rep --build lbvh --rebuild --steps 60 --opt tlas_after_build=$t
  done
done
