#!/bin/bash
# r05 session 14: C5 rebuild with a high-priority scene stream; C2 threshold x leaf_early; occupancy after leaf_early
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05s14; mkdir -p $O
export TMPDIR=/tmp
one() {   # name args...
  local name=$1; shift 1
  timeout -k 10 300 python3 bench.py "$@" --no-cpu-baseline > $O/$name.log 2>&1 || { echo "fail $name"; tail -5 $O/$name.log; exit 1; }
  python3 - $O/$name.log $name <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().split("\n")[-1])
print(f"{sys.argv[2]:18s} lanes {d['config']['overlap_lanes']} ms/frame {d['ms_per_step']:.4f} lat {d['frame_latency_ms_median']:.4f} serial {d['kernel_ms']:.4f}", flush=True)
PY
}
for rep in 1 2; do
  one c5rb_sp0_$rep --config C5 --build lbvh --rebuild --steps 12 --warmup 3
  one c5rb_sp1_$rep --config C5 --build lbvh --rebuild --steps 12 --warmup 3 --pre-opt scene_priority=1
  one c5rb_L3_$rep --config C5 --build lbvh --rebuild --steps 12 --warmup 3 --overlap 3
  for th in 48 56 64; do
    for k in 0 2; do
      one c2_th${th}_le${k}_$rep --steps 100 --threshold $th --opt leaf_early=$k
    done
  done
done
D=$PWD/real-time-gpu-ray-tracer_amd/lib/librtamd_diag.so
for c in "C2|sah" "C3|sah" "C5|lbvh"; do
  cfg=${c%%|*}; b=${c#*|}
  RTAMD_LIB=$D timeout -k 10 300 python3 scripts/timeline.py --config $cfg --build $b --parts 8 --threshold 0 --out $O/tl_$cfg.npz > $O/tl_$cfg.log 2>&1 || { echo "timeline $cfg failed"; tail -3 $O/tl_$cfg.log; exit 1; }
  grep '^{"tag' $O/tl_$cfg.log | head -1 | python3 -c "
import json,sys; d=json.loads(sys.stdin.read())
print('$cfg', {k: d[k] for k in ('span_us','cycle_split_refill_interior_leaf_shade','lanes_per_interior_iter','lanes_per_leaf_phase_tlas_blas','lanes_per_shade','interior_iters_per_round','cycles_per_interior_iter','cycles_per_leaf_phase','cycles_per_shade','mean_life_frac')})"
done
