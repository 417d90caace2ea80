#!/bin/bash
# r05 session 10: library lanes at the box's default 4 hardware queues (lane count, priority), and the diagnostic
# build's per-phase lane occupancy
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05s10; mkdir -p $O
export TMPDIR=/tmp
one() {   # name hwq args...
  local name=$1 q=$2; shift 2
  RTAMD_HWQ=$q timeout -k 10 300 python3 bench.py "$@" --no-cpu-baseline > $O/$name.log 2>&1 || { echo "fail $name"; tail -5 $O/$name.log; exit 1; }
  python3 - $O/$name.log $name $q <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().split("\n")[-1])
print(f"{sys.argv[2]:22s} hwq {sys.argv[3]:>2s} lanes {d['config']['overlap_lanes']} ms/frame {d['ms_per_step']:.4f} lat {d['frame_latency_ms_median']:.4f}", flush=True)
PY
}
for rep in 1 2; do
  one c2_auto_q4_$rep 4 --steps 100
  one c2_L2_q4_$rep 4 --steps 100 --overlap 2
  one c2_L3_q4_$rep 4 --steps 100 --overlap 3
  one c2_L4hi_q4_$rep 4 --steps 100 --opt lane_priority=1
  one c2_auto_q12_$rep 12 --steps 100
  one share_auto_q12_$rep 12 --steps 100 --shard 0/8
  one share_caller_q12_$rep 12 --steps 100 --shard 0/8 --lanes caller
  one share_auto_q4_$rep 4 --steps 100 --shard 0/8
  one share_L4_q4_$rep 4 --steps 100 --shard 0/8 --overlap 4
done
D=$PWD/real-time-gpu-ray-tracer_amd/lib/librtamd_diag.so
for c in "C2|sah" "C3|sah" "C5|lbvh"; do
  cfg=${c%%|*}; b=${c#*|}
  RTAMD_LIB=$D timeout -k 10 300 python3 scripts/timeline.py --config $cfg --build $b --parts 8 --threshold 0 --out $O/tl_$cfg.npz > $O/tl_$cfg.log 2>&1 || { echo "timeline $cfg failed"; tail -3 $O/tl_$cfg.log; exit 1; }
  grep '^{"tag' $O/tl_$cfg.log | head -1 | python3 -c "
import json,sys; d=json.loads(sys.stdin.read())
print('$cfg', {k: d[k] for k in ('span_us','cycle_split_refill_interior_leaf_shade','lanes_per_interior_iter','lanes_per_leaf_phase_tlas_blas','lanes_per_shade','interior_iters_per_round','cycles_per_interior_iter','cycles_per_leaf_phase','cycles_per_shade','mean_life_frac')})"
done
