#!/bin/bash
# r05 session 30: per-rank shares of the 8-GPU configs (C4: the C3 scene at 1 spp; C5 with and without the per-frame
# rebuild) on one GPU, exactly as rank R of an 8-rank run traces them (bench.py --shard R/8)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05s30; mkdir -p $O
export TMPDIR=/tmp
one() {   # name args...
  local name=$1; shift 1
  timeout -k 10 400 python3 bench.py "$@" --no-cpu-baseline > $O/$name.log 2>&1 || { echo "fail $name"; tail -5 $O/$name.log; exit 1; }
  python3 - $O/$name.log $name <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().split("\n")[-1])
print(f"{sys.argv[2]:18s} lanes {d['config']['overlap_lanes']} ms/frame {d['ms_per_step']:.4f} lat {d['frame_latency_ms_median']:.4f} serial {d['kernel_ms']:.4f} Mrays/s {d['value']:.0f}", flush=True)
PY
}
for r in 0 3 6; do
  one c4_s${r} --config C4 --steps 100 --shard $r/8
  one c5_s${r} --config C5 --build lbvh --steps 24 --warmup 4 --shard $r/8
  one c5rb_s${r} --config C5 --build lbvh --rebuild --steps 24 --warmup 4 --shard $r/8
done
