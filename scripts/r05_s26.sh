#!/bin/bash
# r05 session 26: non-temporal RGBA8 stores (keep the frame out of L2) on C2 / C3 / the 1/8 share
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05s26; mkdir -p $O
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
for rep in 1 2 3; do
  for nt in 0 1; do
    one c2_nt${nt}_$rep --steps 100 --opt nt_store=$nt
    one c2ser_nt${nt}_$rep --steps 40 --overlap 1 --opt nt_store=$nt
    one c3_nt${nt}_$rep --config C3 --steps 40 --opt nt_store=$nt
  done
done
