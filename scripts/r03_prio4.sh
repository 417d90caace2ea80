#!/bin/bash
# Study (4): lanes on new normal-priority streams (off the null stream) with 12 hardware queues per process,
# against the current defaults (null stream + new streams, 4 queues), on the full-frame workloads.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/prio4; mkdir -p $OUT
for rep in 1 2; do
for base in "C2 --steps 100" "C3 --steps 40" "C4 --steps 100" "C2 --build lbvh --steps 100" "C2 --build lbvh --rebuild --steps 100" "C5 --build lbvh --rebuild --steps 12" "C5 --build lbvh --steps 12"; do
for var in "def" "q12" "q12p0" "q12pm1"; do
  case $var in def) env=""; pr="";; q12) env="RTAMD_HWQ=12"; pr="";; q12p0) env="RTAMD_HWQ=12"; pr="--lane-priority 0";;
               q12pm1) env="RTAMD_HWQ=12"; pr="--lane-priority -1";; esac
  tag=$(echo "$base $var" | tr ' /' '__' | tr -d -)
  env $env timeout -k 10 300 python3 bench.py --config $base $pr --no-cpu-baseline > $OUT/${tag}_$rep.log 2>&1 || { echo "fail $base $var"; tail -3 $OUT/${tag}_$rep.log; exit 1; }
  echo "$base [$var] rep $rep: $(grep -o '"ms_per_step": [0-9.]*' $OUT/${tag}_$rep.log)"
done; done; done
