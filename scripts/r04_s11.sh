#!/bin/bash
# Round 4 step 11: conservative slab with unwidened ordering; LBVH chunk/Karras LDS staging; C5 grids
set -o pipefail
O=gpurun_out/r04s11; mkdir -p $O
export TMPDIR=/tmp
L=$PWD/real-time-gpu-ray-tracer_amd/lib
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_lbvh.py tests/test_gpu_group.py \
  tests/test_gpu_parity.py > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 200 python -u scripts/rebuild_alone.py --config C5 > $O/alone.log 2>&1 || exit 1
tail -1 $O/alone.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/kst_alone -o run --output-format csv -- python -u scripts/rebuild_alone.py \
  --config C5 > $O/kst_alone.log 2>&1 || exit 1
for v in default oldthr; do
  if [ $v = default ]; then lib=""; else lib=$L/librtamd_$v.so; fi
  RTAMD_LIB=$lib timeout -k 10 400 python -u scripts/parity_report.py --configs C2,C3,C5 --frames 0,37 \
    --modes fast_compat+wide=0,fast_compat --out $O/parity_$v.json > $O/parity_$v.log 2>&1 || exit 1
  python3 -c "
import json
for c in json.load(open('$O/parity_$v.json'))['cases']: print('$v', c['config'],c['frame'],c['mode'],c['outliers_gt1'],c['float_ne'],c['max_lsb'])"
done
for args in "--rebuild --opt grid_pct=100" "--rebuild --opt grid_pct=100 --opt blas_sets=3" "--opt grid_pct=100" ""; do
  tag=$(echo "x$args" | tr -d ' -' | tr '=' '_')
  timeout -k 10 300 python -u bench.py --config C5 --build lbvh --steps 12 --warmup 3 --no-cpu-baseline $args \
    > $O/c5_$tag.log 2>&1 || exit 1
  grep '^{' $O/c5_$tag.log | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('c5 $tag', d['ms_per_step'], d['kernel_ms'])"
done
