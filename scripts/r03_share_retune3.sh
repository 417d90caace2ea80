#!/bin/bash
# Share grids for N = 2 and 4 (rank 0's share, 8 lanes off the null stream, 24 queues as with a communicator).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/share_retune3; mkdir -p $OUT
for sh in "C2 --shard 0/2" "C2 --shard 1/4" "C4 --shard 0/2" "C4 --shard 1/4"; do
for g in 0 20 25 35; do
  o=""; [ "$g" != 0 ] && o="--opt grid_pct=$g"
  tag=$(echo "$sh $g" | tr ' /:' '___' | tr -d -)
  RTAMD_HWQ=24 timeout -k 10 300 python3 bench.py --config $sh $o --steps 200 --no-cpu-baseline > $OUT/$tag.log 2>&1 || { echo "fail $sh $g"; tail -3 $OUT/$tag.log; exit 1; }
  echo "$sh [grid_pct $g]: $(grep -o '"ms_per_step": [0-9.]*' $OUT/$tag.log)"
done; done
