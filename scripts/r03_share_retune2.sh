#!/bin/bash
# Share grids (8 lanes, every lane off the null stream): grid_pct 15 (auto) / 20 / 25 / 30 at 12 and 24 queues.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/share_retune2; mkdir -p $OUT
for sh in "C2 --shard 0/8" "C2 --shard 4/8" "C4 --shard 2/8" "C4 --shard 6/8"; do
for var in "0:12" "20:12" "25:12" "30:12" "0:24" "20:24" "25:24"; do
  IFS=: read -r g q <<< "$var"
  o=""; [ "$g" != 0 ] && o="--opt grid_pct=$g"
  tag=$(echo "$sh $var" | tr ' /:' '___' | tr -d -)
  RTAMD_HWQ=$q timeout -k 10 300 python3 bench.py --config $sh $o --steps 200 --no-cpu-baseline > $OUT/$tag.log 2>&1 || { echo "fail $sh $var"; tail -3 $OUT/$tag.log; exit 1; }
  echo "$sh [grid_pct $g hwq $q]: $(grep -o '"ms_per_step": [0-9.]*' $OUT/$tag.log)"
done; done
