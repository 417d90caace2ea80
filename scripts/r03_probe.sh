#!/bin/bash
# round-3 probes: GPU tests, warm-up dependence of serialised launches, critical path of the heaviest unit
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/probe
mkdir -p $OUT
run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "=== $name: $*"
  timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -3 "$OUT/$name.log" | cut -c1-600
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
}
[ -z "$NO_TESTS" ] && run gpu_tests 600 python -u -m pytest tests -m gpu -x -q -rf --timeout 120 --timeout-method thread ${TEST_ARGS:-}
for w in ${WARMUPS:-10 2000}; do
  run warm_C2_$w 300 python bench.py --overlap 1 --warmup $w --steps 100 --no-cpu-baseline
done
for w in ${WARMUPS_C3:-5 300}; do
  run warm_C3_$w 300 python bench.py --config C3 --overlap 1 --warmup $w --steps 60 --no-cpu-baseline
done
[ -z "$NO_CP" ] && run critical_C2 300 python scripts/critical_path.py
exit 0
