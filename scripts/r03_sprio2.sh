#!/bin/bash
# Study (2): lanes on new normal-priority streams + 12 hardware queues, with and without the scene stream at
# high priority, on the per-frame rebuild workloads (and the plain frames, for a universal default).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/sprio2; mkdir -p $OUT
for rep in 1 2; do
for base in "C5 --build lbvh --rebuild --steps 12" "C2 --build lbvh --rebuild --steps 100" "C2 --build lbvh --steps 100" "C2 --steps 100" "C3 --steps 40"; do
for var in "def" "q12p0" "q12p0sp"; do
  case $var in def) env=""; o="";; q12p0) env="RTAMD_HWQ=12"; o="--lane-priority 0";;
               q12p0sp) env="RTAMD_HWQ=12"; o="--lane-priority 0 --pre-opt scene_priority=-1";; esac
  tag=$(echo "$base $var" | tr ' /' '__' | tr -d -)
  env $env timeout -k 10 300 python3 bench.py --config $base $o --no-cpu-baseline > $OUT/${tag}_$rep.log 2>&1 || { echo "fail $base $var"; tail -3 $OUT/${tag}_$rep.log; exit 1; }
  echo "$base [$var] rep $rep: $(grep -o '"ms_per_step": [0-9.]*' $OUT/${tag}_$rep.log)"
done; done; done
