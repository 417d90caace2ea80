#!/bin/bash
# r05 session 15: refill threshold re-tuned under leaf_early (multi-segment configs)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05s15; mkdir -p $O
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
  for th in 24 32 40 48 56; do
    one c3_th${th}_$rep --config C3 --steps 40 --threshold $th
    one c5_th${th}_$rep --config C5 --build lbvh --steps 12 --warmup 3 --threshold $th
  done
  for k in 8 12 16; do
    one c3_th32_le${k}_$rep --config C3 --steps 40 --threshold 32 --opt leaf_early=$k
    one c5_th32_le${k}_$rep --config C5 --build lbvh --steps 12 --warmup 3 --threshold 32 --opt leaf_early=$k
  done
done
