#!/bin/bash
# Round 4 step 21: the rebuild's gather on an auxiliary stream beside the tree phase
set -o pipefail
O=gpurun_out/r04s21; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_lbvh.py tests/test_gpu_group.py \
  tests/test_gpu_configs.py > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for v in 1 0; do
  timeout -k 10 200 python -u scripts/rebuild_alone.py --config C5 --opt split_gather=$v > $O/alone_$v.log 2>&1 || exit 1
  tail -1 $O/alone_$v.log
done
for rep in 1 2; do
for v in 1 0; do
  timeout -k 10 300 python -u bench.py --config C5 --build lbvh --rebuild --steps 12 --warmup 3 --no-cpu-baseline --opt split_gather=$v \
    > $O/c5_${v}_$rep.log 2>&1 || exit 1
  grep '^{' $O/c5_${v}_$rep.log | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('c5 rebuild split_gather=$v', d['ms_per_step'])"
done
done
