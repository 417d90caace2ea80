#!/bin/bash
# r05 session 28: cold triangle records on GPU-built scenes (one dependent HBM round trip less per shaded triangle hit)
# for C5 with trees built once and with the per-frame rebuild, and C2 on GPU trees
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05s28; mkdir -p $O
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
  for c in 0 1; do
    one c5_cold${c}_$rep --config C5 --build lbvh --steps 12 --warmup 3 --pre-opt cold_records=$c
    one c5ser_cold${c}_$rep --config C5 --build lbvh --steps 6 --warmup 2 --overlap 1 --pre-opt cold_records=$c
    one c5rb_cold${c}_$rep --config C5 --build lbvh --rebuild --steps 12 --warmup 3 --pre-opt cold_records=$c
    one c2l_cold${c}_$rep --build lbvh --steps 100 --pre-opt cold_records=$c
  done
done
