#!/bin/bash
# r05 session 48: C3 claim-order options on the final library (reorder period, longest-path unit costs)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05s48; mkdir -p $O
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
  one c3_def_$rep --config C3 --steps 40
  one c3_p2_$rep --config C3 --steps 40 --opt reorder_period=2
  one c3_cmax_$rep --config C3 --steps 40 --opt cost_max=1
  one c3_p1_$rep --config C3 --steps 40 --opt reorder_period=1
done
