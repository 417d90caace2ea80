#!/bin/bash
# Stack overflow rows in HBM (default) vs lane-swizzled scratch (librtamd_scr.so): GPU tests, C2/C3 A/B,
# and a WRITE_SIZE pass of each (serialised launches)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/gs
mkdir -p $OUT
export TMPDIR=/tmp
step() { local name=$1 to=$2; shift 2; echo "=== $name"; timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "rc=$rc"; tail -3 "$OUT/$name.log" | cut -c1-400; [ $rc -eq 0 ] || exit $rc; }
[ -z "$NO_TESTS" ] && step tests 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 120 --timeout-method thread
rm -f gpurun_out/ab.jsonl
step ab_c2 900 bash scripts/ab_libs.sh 3 "scr=librtamd_scr.so new=default"
step ab_c3 600 bash scripts/ab_libs.sh 1 "scr=librtamd_scr.so new=default" --config C3 --steps 40
cp gpurun_out/ab.jsonl $OUT/ab.jsonl
for v in new scr; do
  lib=librtamd.so; [ $v = scr ] && lib=librtamd_scr.so
  RTAMD_LIB=$PWD/real-time-gpu-ray-tracer_amd/lib/$lib step ws_$v 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/ws_$v -o run --output-format csv -- \
      python3 bench.py --steps 5 --warmup 2 --overlap 1 --no-cpu-baseline --clock-warmup 0
done
exit 0
