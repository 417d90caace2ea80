#!/bin/bash
# C5 (LBVH, per-frame rebuild) with instance groups: bench line + rocprofv3 kernel stats
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/c5prof
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/stats -o run --output-format csv -- \
    python3 bench.py --config C5 --build lbvh --rebuild --steps 8 --warmup 2 --no-cpu-baseline --clock-warmup 0 > $OUT/c5.log 2>&1
echo "c5 rc=$?"
tail -1 $OUT/c5.log | cut -c1-300
