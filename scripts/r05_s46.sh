#!/bin/bash
# r05 session 46: run-to-run spread of the final library on one box — the driver's command five times, C5 with the
# per-frame rebuild three times
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05s46; mkdir -p $O
export TMPDIR=/tmp
one() {   # name args...
  local name=$1; shift 1
  timeout -k 10 400 python3 bench.py "$@" > $O/$name.log 2>&1 || { echo "fail $name"; tail -5 $O/$name.log; exit 1; }
  python3 - $O/$name.log $name <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().split("\n")[-1])
print(f"{sys.argv[2]:14s} ms/frame {d['ms_per_step']:.4f} value {d['value']:.0f} frac {d['roofline']['frac']:.3f} traffic {d['roofline'].get('traffic')}", flush=True)
PY
}
for rep in 1 2 3 4 5; do one driver_$rep --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline; done
for rep in 1 2 3; do one c5rb_$rep --config C5 --build lbvh --rebuild --steps 12 --warmup 3 --no-cpu-baseline; done
