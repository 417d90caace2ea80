#!/bin/bash
# r05 session 49: C5 with trees built once — lane count (library lanes, "overlap" 3..6; auto = 4)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05s49; mkdir -p $O
export TMPDIR=/tmp
one() {   # name args...
  local name=$1; shift 1
  timeout -k 10 300 python3 bench.py "$@" --no-cpu-baseline > $O/$name.log 2>&1 || { echo "fail $name"; tail -5 $O/$name.log; exit 1; }
  python3 - $O/$name.log $name <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().split("\n")[-1])
print(f"{sys.argv[2]:18s} lanes {d['config']['overlap_lanes']} ms/frame {d['ms_per_step']:.4f} lat {d['frame_latency_ms_median']:.4f}", flush=True)
PY
}
for rep in 1 2; do
  one c5_auto_$rep --config C5 --build lbvh --steps 16 --warmup 4
  for L in 3 5 6; do one c5_l${L}_$rep --config C5 --build lbvh --steps 16 --warmup 4 --overlap $L; done
done
