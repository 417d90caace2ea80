#!/bin/bash
# GPU-box check: smoke -> gpu tests -> bench -> rocprofv3 kernel stats.
# Stops at the first step that faults, aborts or times out (exit codes other than 0/1).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "=== $name: $*" | tee -a gpurun_out/summary.log
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a gpurun_out/summary.log
  tail -5 "gpurun_out/$name.log" | tee -a gpurun_out/summary.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
STEPS=${STEPS:-smoke,tests,bench,prof}
[[ $STEPS == *smoke* ]] && run smoke 400 python -c "import __graft_entry__ as g; g.smoke()"
[[ $STEPS == *tests* ]] && run gpu_tests 900 python -u -m pytest ${TEST_ARGS:-tests} -m gpu -v -rf --timeout 120 --timeout-method thread
[[ $STEPS == *ab* ]] && run ab 600 python scripts/ab_kernels.py ${AB_ARGS:-grid:kernel=0 p8:kernel=1,threshold=8 p16:kernel=1,threshold=16 p24:kernel=1,threshold=24 p32:kernel=1,threshold=32 p48:kernel=1,threshold=48}
[[ $STEPS == *timeline* ]] && run timeline 300 python scripts/timeline.py ${TL_ARGS:-}
[[ $STEPS == *bench* ]] && run bench 600 python bench.py
if [[ $STEPS == *prof* ]]; then
  export TMPDIR=/tmp
  run prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline
fi
if [[ $STEPS == *pmc* ]]; then
  KSUB=${KSUB:-"dev_fast::render_persistent_kernel<false"}
  run pmc 800 bash scripts/pmc_passes.sh gpurun_out/pmc "$KSUB" -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline
fi
[[ $STEPS == *list* ]] && run counters 120 rocprofv3 -L
exit 0
