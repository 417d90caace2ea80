#!/bin/bash
# Share settings re-checked with every lane off the null stream: lanes x grid_pct x hardware queues, C2 0/8 and C4 2/8.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/share_retune; mkdir -p $OUT
for sh in "C2 --shard 0/8" "C4 --shard 2/8"; do
for var in "8:0:12" "8:0:16" "8:10:12" "8:20:12" "6:20:12" "6:0:12" "8:0:24"; do
  IFS=: read -r L g q <<< "$var"
  o="--overlap $L"; [ "$g" != 0 ] && o="$o --opt grid_pct=$g"
  tag=$(echo "$sh $var" | tr ' /:' '___' | tr -d -)
  RTAMD_HWQ=$q timeout -k 10 300 python3 bench.py --config $sh $o --steps 200 --no-cpu-baseline > $OUT/$tag.log 2>&1 || { echo "fail $sh $var"; tail -3 $OUT/$tag.log; exit 1; }
  echo "$sh [lanes $L grid_pct $g hwq $q]: $(grep -o '"ms_per_step": [0-9.]*' $OUT/$tag.log)"
done; done
