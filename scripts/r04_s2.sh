#!/bin/bash
# Round-4 session 2: which FAST arithmetic makes the parity outliers (variants of the FAST kernel: IEEE division /
# 1/sqrt in primitives + shading, with / without FMA contraction), what each costs; the fake-RCCL world > 1 test.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r04s2
mkdir -p $OUT
export TMPDIR=/tmp
run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "=== $name"
  timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "rc=$rc"; tail -1 "$OUT/$name.log" | cut -c1-300
  if [ $rc -ne 0 ]; then tail -15 "$OUT/$name.log"; exit $rc; fi
}
run fake_rccl 400 python -u -m pytest tests/test_gpu_fake_rccl.py tests/test_gpu_group.py tests/test_gpu_lbvh.py -x -q -rf --timeout 300 --timeout-method thread
LIBDIR=$PWD/real-time-gpu-ray-tracer_amd/lib
for v in default ieee1 ieee2 ieee1c nocontract; do
  if [ $v = default ]; then L=$LIBDIR/librtamd.so; else L=$LIBDIR/librtamd_$v.so; fi
  RTAMD_LIB=$L run parity_$v 600 python3 -u scripts/parity_report.py --configs C2,C3 --modes bench,fast_compat,fast_compat_binary --out $OUT/parity_$v.json
  RTAMD_LIB=$L run bench_c2_$v 300 python3 bench.py --steps 100 --no-cpu-baseline
  RTAMD_LIB=$L run bench_c3_$v 300 python3 bench.py --config C3 --steps 40 --no-cpu-baseline
done
exit 0
