#!/bin/bash
# Round 4 step 13: C5 with the reference's visit order (binary node pairs) on the GPU LBVH trees: parity + cost
set -o pipefail
O=gpurun_out/r04s13; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/parity_report.py --configs C5 --frames 0,37 --modes lbvh+wide=0,lbvh+wide=0+fast_math=1,lbvh+fast_math=1 \
  --out $O/parity_c5_binary.json > $O/parity_c5_binary.log 2>&1 || exit 1
grep '"mode"' $O/parity_c5_binary.log | cut -c1-175
for args in "--rebuild --opt wide=0" "--opt wide=0" "--rebuild" ""; do
  tag=$(echo "x$args" | tr -d ' -' | tr '=' '_')
  timeout -k 10 300 python -u bench.py --config C5 --build lbvh --steps 12 --warmup 3 --no-cpu-baseline $args \
    > $O/c5_$tag.log 2>&1 || exit 1
  grep '^{' $O/c5_$tag.log | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('c5 $tag', d['ms_per_step'], d['kernel_ms'])"
done
