#!/bin/bash
# r05 session 22: BLAS Morton sort in three 10-bit onesweep passes (sort10) against HEAD (r05b): LBVH tests, C5 rebuild
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05s22; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_lbvh.py tests/test_gpu_group.py tests/test_gpu_configs.py -m gpu -x -q -rf --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/tests.log; [ $rc -ne 0 ] && exit $rc
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
for rep in 1 2 3; do
  for v in sort10 r05b; do
    one c5rb_$rep $v --config C5 --build lbvh --rebuild --steps 12 --warmup 3
  done
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/ks -o run --output-format csv -- \
    python3 bench.py --config C5 --build lbvh --rebuild --steps 6 --warmup 2 --overlap 1 --no-cpu-baseline > $O/ks.log 2>&1 || { tail -5 $O/ks.log; exit 1; }
f=$(find $O/ks -name '*kernel_stats.csv' | head -1)
python3 - "$f" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "render_persistent" in r["Name"]: continue
    if float(r["AverageNs"]) * int(r["Calls"]) < 2e6: continue
    print(f'{int(r["Calls"]):6d} {float(r["AverageNs"])/1000:9.1f} us  {r["Name"][:100]}')
PY
find $O/ks -name '*kernel_trace.csv' -delete
