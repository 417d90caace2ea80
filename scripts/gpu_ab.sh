#!/bin/bash
# GPU-box: targeted GPU tests, then an in-process A/B of kernel options (scripts/ab_kernels.py).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "${KEXPR:-}" > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/gpu_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 400 python -u scripts/ab_kernels.py --config ${CONFIG:-C2} --rounds ${ROUNDS:-4} --frames 10 ${AB:-base:build=sah,reorder=0,threshold=8 lpt:build=sah,reorder=1,threshold=8} > gpurun_out/ab.log 2>&1
rc=$?; echo "ab rc=$rc"; cat gpurun_out/ab.log
exit $rc
