#!/bin/bash
# Whole frame, lanes off the null stream, 12 queues: lanes x grid_pct on C2, then the candidates on C3 / C4 /
# C2-LBVH / C5 against the defaults.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/lanes_new2; mkdir -p $OUT
run() { tag=$1; shift; RTAMD_HWQ=12 timeout -k 10 300 python3 bench.py "$@" --no-cpu-baseline > $OUT/$tag.log 2>&1 || { echo "fail $tag"; tail -3 $OUT/$tag.log; exit 1; }
        echo "$tag: $(grep -o '"ms_per_step": [0-9.]*' $OUT/$tag.log)"; }
for rep in 1 2; do
run c2_def_$rep --config C2 --steps 100
for lg in 4:30 4:35 4:40 4:45 5:30 5:40 6:25 6:33; do IFS=: read -r L g <<< "$lg"
  run c2_l${L}_g${g}_$rep --config C2 --steps 100 --lane-priority 0 --overlap $L --opt grid_pct=$g; done
done
for cfg in "C3 --steps 40" "C4 --steps 100" "C2 --build lbvh --steps 100" "C5 --build lbvh --steps 12"; do
  t=$(echo $cfg | cut -d' ' -f1)$(echo "$cfg" | grep -q lbvh && echo _lbvh)
  for rep in 1 2; do
  run ${t}_def_$rep --config $cfg
  run ${t}_l4_g40_$rep --config $cfg --lane-priority 0 --overlap 4 --opt grid_pct=40
  run ${t}_l5_g30_$rep --config $cfg --lane-priority 0 --overlap 5 --opt grid_pct=30
  done
done
