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
[[ $STEPS == *tests* ]] && run gpu_tests 900 python -m pytest tests -m gpu -q -rf
[[ $STEPS == *ab* ]] && run ab 600 python scripts/ab_kernels.py ${AB_ARGS:-grid:kernel=0 p8:kernel=1,threshold=8 p16:kernel=1,threshold=16 p24:kernel=1,threshold=24 p32:kernel=1,threshold=32 p48:kernel=1,threshold=48}
[[ $STEPS == *bench* ]] && run bench 600 python bench.py
if [[ $STEPS == *prof* ]]; then
  export TMPDIR=/tmp
  run prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline
fi
if [[ $STEPS == *pmc* ]]; then
  export TMPDIR=/tmp
  BENCH="python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline"
  run pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o run --output-format csv -- $BENCH
  run pmc_write 600 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write -o run --output-format csv -- $BENCH
  run pmc_sq 600 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE -d gpurun_out/pmc_sq -o run --output-format csv -- $BENCH
  run pmc_tcc 600 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d gpurun_out/pmc_tcc -o run --output-format csv -- $BENCH
  python3 scripts/pmc_summary.py gpurun_out/pmc_summary.json "dev_fast::render_kernel<false>" gpurun_out/pmc_fetch gpurun_out/pmc_write gpurun_out/pmc_sq gpurun_out/pmc_tcc > gpurun_out/pmc_summary.log 2>&1
fi
[[ $STEPS == *list* ]] && run counters 120 rocprofv3 -L
exit 0
