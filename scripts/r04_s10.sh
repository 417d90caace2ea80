#!/bin/bash
# Round 4 step 10: conservative slab (RT_SLAB_CONS) parity + cost; C5 rebuild with three BLAS sets / full grids
set -o pipefail
O=gpurun_out/r04s10; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_lbvh.py tests/test_gpu_group.py \
  tests/test_gpu_parity.py > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -u scripts/parity_report.py --configs C5 --frames 0 --modes fast_compat+wide=0,fast_compat \
  --out $O/parity_c5.json > $O/parity_c5.log 2>&1 || exit 1
grep '"mode"' $O/parity_c5.log | cut -c1-160
timeout -k 10 400 python -u scripts/parity_report.py --configs C2,C3 --modes fast_compat+wide=0,fast_compat,bench \
  --out $O/parity_c23.json > $O/parity_c23.log 2>&1 || exit 1
grep '"mode"' $O/parity_c23.log | cut -c1-160
for args in "--opt blas_sets=3" "--opt blas_sets=3 --opt grid_pct=100" "--opt grid_pct=100" ""; do
  tag=$(echo "x$args" | tr -d ' -' | tr '=' '_')
  timeout -k 10 300 python -u bench.py --config C5 --build lbvh --rebuild --steps 12 --warmup 3 --no-cpu-baseline $args \
    > $O/c5_$tag.log 2>&1 || exit 1
  grep '^{' $O/c5_$tag.log | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('c5 $tag', d['ms_per_step'])"
done
OPT=lib VALS="default nocons" REPS=2 CASES="c2_100|--steps 100;share8|--steps 100 --shard 0/8;c3|--config C3 --steps 40" \
  timeout -k 10 600 bash scripts/r04_ab.sh r04s10/ab
