#!/bin/bash
# Round-4 session 1: GPU tests with the new ones, full-frame parity numbers of the benched configuration (default
# library and the parallel-axis-branch variant), the driver's bench command, a 100-step bench line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r04s1
mkdir -p $OUT
export TMPDIR=/tmp
run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "=== $name"
  timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "rc=$rc"; tail -2 "$OUT/$name.log" | cut -c1-300
  if [ $rc -ne 0 ]; then tail -15 "$OUT/$name.log"; exit $rc; fi
}
run tests 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread
run parity 600 python3 -u scripts/parity_report.py --out $OUT/parity_default.json --save-diff $OUT/diff_default
RTAMD_LIB=$PWD/real-time-gpu-ray-tracer_amd/lib/librtamd_tiny.so run parity_tiny 600 \
    python3 -u scripts/parity_report.py --modes bench,fast_compat --out $OUT/parity_tiny.json --save-diff $OUT/diff_tiny
run bench_driver 300 python3 bench.py --gpus 1 --steps 20 --warmup 5
run bench_100 300 python3 bench.py --steps 100 --no-cpu-baseline
exit 0
