#!/bin/bash
# r05 session 35: frame unit shape (option "unit_shape": 8x8, 16x4, 32x2, 64x1) against C2 write traffic
# (verdict r4 item 8) and ms/frame on C2 / C2 serialised / C3
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05s35; mkdir -p $O
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
for us in 3 4 5 6; do
  PMC_STEPS=5 timeout -k 10 400 bash scripts/pmc_tagged.sh $O/pmc_us$us -- --opt unit_shape=$us > $O/pmc_us$us.log 2>&1 || { echo "pmc fail $us"; tail -5 $O/pmc_us$us.log; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/pmc_us$us/summary.json')); print('us$us write MB', round(d['write_bytes_per_launch']/1e6,2), 'fetch MB', round(d['fetch_bytes_per_launch_corrected']/1e6,2))"
  rm -rf $O/pmc_us$us/pass*
done
for rep in 1 2; do
  for us in 3 4 5 6; do
    one c2_us${us}_$rep --steps 100 --opt unit_shape=$us
    one c2ser_us${us}_$rep --steps 40 --overlap 1 --opt unit_shape=$us
    one c3_us${us}_$rep --config C3 --steps 40 --opt unit_shape=$us
  done
done
