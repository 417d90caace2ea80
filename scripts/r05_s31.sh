#!/bin/bash
# r05 session 31: C5 per-rank share (1/8) with the per-frame rebuild: lanes 1..8
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05s31; mkdir -p $O
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
  for L in 1 2 3 4; do
    one c5rb_s0_L${L}_$rep --config C5 --build lbvh --rebuild --steps 24 --warmup 4 --shard 0/8 --overlap $L
  done
  one c5rb_s0_auto_$rep --config C5 --build lbvh --rebuild --steps 24 --warmup 4 --shard 0/8
done
timeout -k 10 300 python3 scripts/rebuild_alone.py --config C5 > $O/alone.log 2>&1 && tail -3 $O/alone.log
