#!/bin/bash
# Round 4, session step 8: C5 compat residual under conservative slab variants; C5 rebuild kernels alone (serial)
set -o pipefail
O=gpurun_out/r04s8; mkdir -p $O
L=real-time-gpu-ray-tracer_amd/lib
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_lbvh.py tests/test_gpu_group.py \
  > $O/tests_lbvh.log 2>&1 || exit 1
for v in pad tiny padtiny; do
  RTAMD_LIB=$L/librtamd_$v.so timeout -k 10 300 python -u scripts/parity_report.py --configs C5 --frames 0 \
    --modes fast_compat+wide=0,fast_compat --out $O/parity_$v.json > $O/parity_$v.log 2>&1 || exit 1
done
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --config C5 --build lbvh --rebuild --overlap 1 --opt blas_double=0 --steps 10 --warmup 3 \
  --no-cpu-baseline > $O/bench_c5_serial.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_serial -o run -- python -u bench.py --config C5 --build lbvh \
  --rebuild --overlap 1 --opt blas_double=0 --steps 10 --warmup 3 --no-cpu-baseline > $O/prof_serial.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --config C5 --build lbvh --rebuild --steps 10 --warmup 3 --no-cpu-baseline > $O/bench_c5_default.log 2>&1
