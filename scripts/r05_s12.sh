#!/bin/bash
# r05 session 12: leaf_early K for the multi-segment configs, defaults check at the box's default 4 queues
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05s12; mkdir -p $O
export TMPDIR=/tmp
one() {   # name args...
  local name=$1; shift 1
  timeout -k 10 300 python3 bench.py "$@" --no-cpu-baseline > $O/$name.log 2>&1 || { echo "fail $name"; tail -5 $O/$name.log; exit 1; }
  python3 - $O/$name.log $name <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().split("\n")[-1])
print(f"{sys.argv[2]:18s} hwq {d['config']['hw_queues']:>2d} lanes {d['config']['overlap_lanes']} ms/frame {d['ms_per_step']:.4f} lat {d['frame_latency_ms_median']:.4f} serial {d['kernel_ms']:.4f} frac {d['roofline']['frac']:.3f}", flush=True)
PY
}
for rep in 1 2; do
  for k in 8 12 16 24 32; do
    one c3_le${k}_$rep --config C3 --steps 40 --opt leaf_early=$k
    one c5_le${k}_$rep --config C5 --build lbvh --steps 12 --warmup 3 --opt leaf_early=$k
  done
  one c5rb_auto_$rep --config C5 --build lbvh --rebuild --steps 12 --warmup 3
  one c2_auto_$rep --steps 100
  one c2w_auto_$rep --steps 20 --warmup 5
  one c4_auto_$rep --config C4 --steps 100
  one share_auto_$rep --steps 100 --shard 0/8
done
