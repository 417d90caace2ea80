#!/bin/bash
# r05 session 9: library-owned lanes ("overlap" -1) against caller lanes, at the default 4 and at 12 hardware queues
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05s9; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_edges.py -k null_stream -q --timeout 200 --timeout-method thread > $O/null.log 2>&1; echo "null rc=$?"; tail -1 $O/null.log
for rep in 1 2; do
for q in 4 12; do
  for mode in library caller; do
    for c in "c2|--steps 100" "c2w|--steps 20 --warmup 5" "share|--steps 100 --shard 0/8" "c3|--config C3 --steps 40"; do
      name=${c%%|*}; args=${c#*|}
      RTAMD_HWQ=$q timeout -k 10 300 python3 bench.py $args --lanes $mode --no-cpu-baseline > $O/${name}_${mode}_q${q}_$rep.log 2>&1 || { echo "fail $name $mode $q"; tail -5 $O/${name}_${mode}_q${q}_$rep.log; exit 1; }
      python3 - $O/${name}_${mode}_q${q}_$rep.log $name $mode $q <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().split("\n")[-1])
print(f"{sys.argv[2]:6s} {sys.argv[3]:8s} hwq {sys.argv[4]:>2s} lanes {d['config']['overlap_lanes']} ms/frame {d['ms_per_step']:.4f} lat {d['frame_latency_ms_median']:.4f}", flush=True)
PY
    done
  done
done
done
# per-phase lane occupancy of the diagnostic build (timeline words 16-19), serialised frame, the library's defaults
D=$PWD/real-time-gpu-ray-tracer_amd/lib/librtamd_diag.so
for c in "C2|sah" "C3|sah" "C5|lbvh"; do
  cfg=${c%%|*}; b=${c#*|}
  RTAMD_LIB=$D timeout -k 10 300 python3 scripts/timeline.py --config $cfg --build $b --parts 8 --threshold 0 --out $O/tl_$cfg.npz > $O/tl_$cfg.log 2>&1 || { echo "timeline $cfg failed"; tail -3 $O/tl_$cfg.log; exit 1; }
  head -1 $O/tl_$cfg.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read())
print('$cfg', {k: d[k] for k in ('span_us','cycle_split_refill_interior_leaf_shade','lanes_per_interior_iter','lanes_per_leaf_phase_tlas_blas','lanes_per_shade','interior_iters_per_round','cycles_per_interior_iter','cycles_per_leaf_phase','cycles_per_shade','mean_life_frac')})"
done
