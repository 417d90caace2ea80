#!/bin/bash
# Round 4 step 25: raw-triangle shading in its own persistent-kernel instance
set -o pipefail
O=gpurun_out/r04s25; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/cold_records_ab.py C2 C5 > $O/cold_ab.log 2>&1 || { tail -5 $O/cold_ab.log; exit 1; }
cat $O/cold_ab.log
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_lbvh.py tests/test_gpu_group.py \
  tests/test_gpu_configs.py tests/test_gpu_golden.py tests/test_gpu_parity.py tests/test_gpu_instances.py > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for v in 0 1; do
  timeout -k 10 200 python -u scripts/rebuild_alone.py --config C5 --pre-opt cold_records=$v > $O/alone_$v.log 2>&1 || { tail -3 $O/alone_$v.log; exit 1; }
  tail -1 $O/alone_$v.log
done
for rep in 1 2; do
for v in 0 1; do
  timeout -k 10 300 python -u bench.py --config C5 --build lbvh --rebuild --steps 12 --warmup 3 --no-cpu-baseline --pre-opt cold_records=$v \
    > $O/c5_${v}_$rep.log 2>&1 || exit 1
  grep '^{' $O/c5_${v}_$rep.log | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('c5 rebuild cold_records=$v', d['ms_per_step'])"
done
done
OPT=lib VALS="default oldfin" REPS=2 CASES="c2_100|--steps 100;c3|--config C3 --steps 40" timeout -k 10 400 bash scripts/r04_ab.sh r04s25/ab
