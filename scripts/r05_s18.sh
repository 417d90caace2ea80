#!/bin/bash
# r05 session 18: drain assist (idle lanes prefetch the stacked nodes of a wave's last tracing lanes) against HEAD
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05s18; mkdir -p $O
export TMPDIR=/tmp
L=$PWD/real-time-gpu-ray-tracer_amd/lib
one() {   # name lib args...
  local name=$1 v=$2; shift 2
  local lib=""; [ $v != default ] && lib=$L/librtamd_$v.so
  RTAMD_LIB=$lib timeout -k 10 300 python3 bench.py "$@" --no-cpu-baseline > $O/${name}_$v.log 2>&1 || { echo "fail $name $v"; tail -5 $O/${name}_$v.log; exit 1; }
  python3 - $O/${name}_$v.log $name $v <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().split("\n")[-1])
print(f"{sys.argv[2]:10s} {sys.argv[3]:8s} ms/frame {d['ms_per_step']:.4f} lat {d['frame_latency_ms_median']:.4f} serial {d['kernel_ms']:.4f}", flush=True)
PY
}
for rep in 1 2; do
  for v in assist r05b; do
    one c5ser_$rep $v --config C5 --build lbvh --steps 6 --warmup 2 --overlap 1
    one c2ser_$rep $v --steps 40 --overlap 1
    one c3ser_$rep $v --config C3 --steps 20 --overlap 1
    one c5_$rep $v --config C5 --build lbvh --steps 12 --warmup 3
    one c2_$rep $v --steps 100
    one c3_$rep $v --config C3 --steps 40
  done
done
for v in assist r05b; do
  RTAMD_LIB=$L/librtamd_$v.so timeout -k 10 300 python3 scripts/timeline.py --config C5 --build lbvh --parts 8 --out $O/tl_C5_$v.npz > $O/tl_C5_$v.log 2>&1 || { echo "timeline $v failed"; tail -3 $O/tl_C5_$v.log; exit 1; }
  grep '^{"tag' $O/tl_C5_$v.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); print('$v', {k: d[k] for k in ('span_us','exhaust_us_p1_p50_p99','drain_us_p50_p99_max','rounds_p50_max','mean_life_frac','kernel_ms_event')})"
  rm -f $O/tl_C5_$v.npz
done
