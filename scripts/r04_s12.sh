#!/bin/bash
# Round 4 step 12: chunk frontier aggregation, big-launch full grid, 3 BLAS sets; FAST vs EXACT on the bench's trees
set -o pipefail
O=gpurun_out/r04s12; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_lbvh.py tests/test_gpu_group.py \
  tests/test_gpu_parity.py > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 200 python -u scripts/rebuild_alone.py --config C5 > $O/alone.log 2>&1 || exit 1
tail -1 $O/alone.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/kst_alone -o run --output-format csv -- python -u scripts/rebuild_alone.py \
  --config C5 > $O/kst_alone.log 2>&1 || exit 1
for args in "--rebuild" ""; do
  tag=$(echo "x$args" | tr -d ' -' | tr '=' '_')
  timeout -k 10 300 python -u bench.py --config C5 --build lbvh --steps 12 --warmup 3 --no-cpu-baseline $args \
    > $O/c5_$tag.log 2>&1 || exit 1
  grep '^{' $O/c5_$tag.log | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('c5 $tag', d['ms_per_step'], d['kernel_ms'])"
done
timeout -k 10 300 python -u scripts/parity_report.py --configs C5 --frames 0,37 --modes lbvh,exact_lbvh --pairs lbvh:exact_lbvh \
  --out $O/parity_c5_trees.json > $O/parity_c5_trees.log 2>&1 || exit 1
grep '"mode"' $O/parity_c5_trees.log | cut -c1-175
timeout -k 10 400 python -u scripts/parity_report.py --configs C2,C3 --frames 0,37 --modes bench,exact_sah --pairs bench:exact_sah \
  --out $O/parity_c23_trees.json > $O/parity_c23_trees.log 2>&1 || exit 1
grep '"mode"' $O/parity_c23_trees.log | cut -c1-175
timeout -k 10 900 python -u -m pytest -q -rf --timeout 600 --timeout-method thread tests/test_gpu_parity_full.py > $O/tests_full.log 2>&1
tail -8 $O/tests_full.log
