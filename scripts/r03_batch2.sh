#!/bin/bash
# GPU tests, LBVH bench lines, C2-LBVH kernel trace, C2 write-breakdown PMC passes
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/b2
mkdir -p $OUT
export TMPDIR=/tmp
step() { local name=$1 to=$2; shift 2; echo "=== $name"; timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "rc=$rc"; tail -2 "$OUT/$name.log" | cut -c1-400; [ $rc -eq 0 ] || exit $rc; }
step gpu_tests 600 python -u -m pytest tests -m gpu -x -q -rf --timeout 120 --timeout-method thread
step c2_lbvh 300 python3 bench.py --build lbvh --no-cpu-baseline
step c2_sah 300 python3 bench.py --no-cpu-baseline
step c5_group 600 python3 bench.py --config C5 --build lbvh --rebuild --steps 12 --warmup 3 --no-cpu-baseline
step kt_lbvh 300 rocprofv3 --kernel-trace -d $OUT/kt_lbvh -o run --output-format csv -- python3 bench.py --build lbvh --steps 40 --warmup 5 --no-cpu-baseline --clock-warmup 0
step pmc_wr 300 rocprofv3 --pmc SQ_INSTS_VMEM_WR SQ_WAVES TCP_TCC_WRITE_REQ_sum TA_FLAT_WRITE_WAVEFRONTS_sum TD_STORE_WAVEFRONT_sum -d $OUT/pmc_wr -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --overlap 1 --no-cpu-baseline --clock-warmup 0
step pmc_ws 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_ws -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --overlap 1 --no-cpu-baseline --clock-warmup 0
