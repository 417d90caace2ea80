#!/bin/bash
# r05 session 45: BLAS quads written by the emission kernel (no collapse pass):
# LBVH GPU tests, the rebuild alone, C5 / C2-LBVH with the per-frame rebuild, against the final library (base)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05s45; mkdir -p $O
export TMPDIR=/tmp
L=$PWD/real-time-gpu-ray-tracer_amd/lib
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_lbvh.py -x -q --timeout 300 --timeout-method thread -m gpu > $O/tests_lbvh.log 2>&1 || { echo "tests fail"; tail -20 $O/tests_lbvh.log; exit 1; }
tail -2 $O/tests_lbvh.log
one() {   # lib name args...
  local v=$1 name=$2; shift 2
  lib=""; [ $v != default ] && lib=$L/librtamd_$v.so
  RTAMD_LIB=$lib timeout -k 10 400 python3 bench.py "$@" --no-cpu-baseline > $O/$name.log 2>&1 || { echo "fail $name"; tail -5 $O/$name.log; exit 1; }
  python3 - $O/$name.log $name <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().split("\n")[-1])
print(f"{sys.argv[2]:22s} ms/frame {d['ms_per_step']:.4f} lat {d['frame_latency_ms_median']:.4f} serial {d['kernel_ms']:.4f}", flush=True)
PY
}
for v in base default; do
  lib=""; [ $v != default ] && lib=$L/librtamd_$v.so
  RTAMD_LIB=$lib timeout -k 10 300 python3 scripts/rebuild_alone.py --config C5 --updates 20 > $O/alone_$v.log 2>&1 || { echo "alone fail"; tail -5 $O/alone_$v.log; exit 1; }
  echo "$v $(tail -1 $O/alone_$v.log)"
done
for rep in 1 2 3; do
  for v in base default; do
    one $v c5rb_${v}_$rep --config C5 --build lbvh --rebuild --steps 12 --warmup 3
    one $v c2lrb_${v}_$rep --build lbvh --rebuild --steps 60
  done
done
