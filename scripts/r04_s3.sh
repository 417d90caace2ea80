#!/bin/bash
# Round-4 session 3: the IEEE-arithmetic FAST kernel as the default: all GPU tests (full-frame parity bars, fake
# RCCL world > 1), the parity report, the driver's bench command and a 100-step line, fast_math beside it.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r04s3
mkdir -p $OUT
export TMPDIR=/tmp
run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "=== $name"
  timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "rc=$rc"; tail -2 "$OUT/$name.log" | cut -c1-300
  if [ $rc -ne 0 ]; then tail -30 "$OUT/$name.log"; exit $rc; fi
}
run tests 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread
run parity 600 python3 -u scripts/parity_report.py --configs C2d1,C2,C3 --modes bench,fast_compat,exact_compat --out $OUT/parity.json
run bench_driver 300 python3 bench.py --gpus 1 --steps 20 --warmup 5
run bench_100 300 python3 bench.py --steps 100 --no-cpu-baseline
run bench_100_fastmath 300 python3 bench.py --steps 100 --no-cpu-baseline --opt fast_math=1
run bench_c3 300 python3 bench.py --config C3 --steps 40 --no-cpu-baseline
run bench_c3_fastmath 300 python3 bench.py --config C3 --steps 40 --no-cpu-baseline --opt fast_math=1
exit 0
