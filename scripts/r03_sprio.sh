#!/bin/bash
# Study: the library's scene stream (per-frame BLAS rebuilds) at high priority (option "scene_priority" -1):
# a high-priority stream takes a hardware queue of its own pool, so it never queues behind a trace lane.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/sprio; mkdir -p $OUT
for rep in 1 2; do
for base in "C5 --build lbvh --rebuild --steps 12" "C2 --build lbvh --rebuild --steps 100" "C2 --build lbvh --steps 100" "C2 --steps 100" "C2 --shard 0/8 --steps 200" "C2 --attach-comm --steps 100"; do
for var in "def" "sp" "spq12"; do
  case $var in def) env=""; o="";; sp) env=""; o="--pre-opt scene_priority=-1";; spq12) env="RTAMD_HWQ=12"; o="--pre-opt scene_priority=-1";; esac
  [ "$var" = spq12 ] && case "$base" in *shard*|*comm*) continue;; esac
  tag=$(echo "$base $var" | tr ' /' '__' | tr -d -)
  env $env timeout -k 10 300 python3 bench.py --config $base $o --no-cpu-baseline > $OUT/${tag}_$rep.log 2>&1 || { echo "fail $base $var"; tail -3 $OUT/${tag}_$rep.log; exit 1; }
  echo "$base [$var] rep $rep: $(grep -o '"ms_per_step": [0-9.]*' $OUT/${tag}_$rep.log)"
done; done; done
