#!/bin/bash
# Round 4 step 26: the builder reads a compact vertex array (36 B per triangle) instead of rt_triangle (88 B)
set -o pipefail
O=gpurun_out/r04s26; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/cold_records_ab.py C2 C5 > $O/cold_ab.log 2>&1 || { tail -5 $O/cold_ab.log; exit 1; }
cat $O/cold_ab.log
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_lbvh.py tests/test_gpu_group.py \
  tests/test_gpu_configs.py tests/test_gpu_golden.py tests/test_gpu_parity.py tests/test_gpu_instances.py > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 200 python -u scripts/rebuild_alone.py --config C5 > $O/alone.log 2>&1 || { tail -3 $O/alone.log; exit 1; }
tail -1 $O/alone.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/kst_alone -o run --output-format csv -- python -u scripts/rebuild_alone.py \
  --config C5 > $O/kst_alone.log 2>&1 || exit 1
for rep in 1 2; do
  timeout -k 10 300 python -u bench.py --config C5 --build lbvh --rebuild --steps 12 --warmup 3 --no-cpu-baseline > $O/c5_$rep.log 2>&1 || exit 1
  grep '^{' $O/c5_$rep.log | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('c5 rebuild', d['ms_per_step'])"
done
