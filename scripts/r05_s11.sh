#!/bin/bash
# r05 session 11: high-priority library lanes at 4 queues on every config; the interior loop's early exit (leaf_early)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05s11; mkdir -p $O
export TMPDIR=/tmp
one() {   # name hwq args...
  local name=$1 q=$2; shift 2
  RTAMD_HWQ=$q timeout -k 10 300 python3 bench.py "$@" --no-cpu-baseline > $O/$name.log 2>&1 || { echo "fail $name"; tail -5 $O/$name.log; exit 1; }
  python3 - $O/$name.log $name $q <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().split("\n")[-1])
print(f"{sys.argv[2]:22s} hwq {sys.argv[3]:>2s} lanes {d['config']['overlap_lanes']} ms/frame {d['ms_per_step']:.4f} lat {d['frame_latency_ms_median']:.4f} serial {d['kernel_ms']:.4f}", flush=True)
PY
}
for rep in 1 2; do
  for pr in 0 1; do
    one c3_p${pr}_q4_$rep 4 --config C3 --steps 40 --opt lane_priority=$pr
    one c5_p${pr}_q4_$rep 4 --config C5 --build lbvh --steps 12 --warmup 3 --opt lane_priority=$pr
    one c5rb_p${pr}_q4_$rep 4 --config C5 --build lbvh --rebuild --steps 12 --warmup 3 --opt lane_priority=$pr
    one share_p${pr}_q4_$rep 4 --steps 100 --shard 0/8 --opt lane_priority=$pr
    one c5rb_p${pr}_q12_$rep 12 --config C5 --build lbvh --rebuild --steps 12 --warmup 3 --opt lane_priority=$pr
  done
  for k in 0 4 8 16; do
    one c2_le${k}_$rep 12 --steps 100 --opt leaf_early=$k
    one c3_le${k}_$rep 12 --config C3 --steps 40 --opt leaf_early=$k
    one c5_le${k}_$rep 12 --config C5 --build lbvh --steps 12 --warmup 3 --opt leaf_early=$k
  done
done
