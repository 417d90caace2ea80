#!/bin/bash
# r05 session 32: auto lanes 2 for rebuild shares — C5 / C4-scene shares with the rebuild, C2-LBVH whole frame with
# the rebuild at 2 / 4 lanes, plus the shares without the rebuild (unchanged: 8 lanes)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05s32; mkdir -p $O
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
  for r in 0 6; do
    one c5rb_s${r}_auto_$rep --config C5 --build lbvh --rebuild --steps 24 --warmup 4 --shard $r/8
  done
  one c2lrb_L2_$rep --build lbvh --rebuild --steps 60 --overlap 2
  one c2lrb_L4_$rep --build lbvh --rebuild --steps 60 --overlap 4
  one c2lrb_auto_$rep --build lbvh --rebuild --steps 60
done
