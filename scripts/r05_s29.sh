#!/bin/bash
# r05 session 29: C5 (trees built once, cold records) refill threshold x leaf_early re-check on the final library
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05s29; mkdir -p $O
export TMPDIR=/tmp
one() {   # name args...
  local name=$1; shift 1
  timeout -k 10 300 python3 bench.py "$@" --no-cpu-baseline > $O/$name.log 2>&1 || { echo "fail $name"; tail -5 $O/$name.log; exit 1; }
  python3 - $O/$name.log $name <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().split("\n")[-1])
print(f"{sys.argv[2]:18s} ms/frame {d['ms_per_step']:.4f} lat {d['frame_latency_ms_median']:.4f} serial {d['kernel_ms']:.4f}", flush=True)
PY
}
for rep in 1 2; do
  one c5_default_$rep --config C5 --build lbvh --steps 12 --warmup 3
  for th in 32 48; do
    one c5_th${th}_$rep --config C5 --build lbvh --steps 12 --warmup 3 --threshold $th
  done
  for le in 8 16 24; do
    one c5_le${le}_$rep --config C5 --build lbvh --steps 12 --warmup 3 --opt leaf_early=$le
  done
  one c3_le16_$rep --config C3 --steps 40 --opt leaf_early=16
  one c3_default_$rep --config C3 --steps 40
done
