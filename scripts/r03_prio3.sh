#!/bin/bash
# Study (3): is it the priority or leaving the null stream?  lanes = [current stream] + new (default),
# all new at priority 0, all new at priority -1.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/prio3; mkdir -p $OUT
for rep in 1 2; do
for base in "C2 --shard 0/8 --steps 200" "C2 --attach-comm --steps 100" "C2 --steps 100" "C5 --build lbvh --rebuild --steps 12" "C2 --build lbvh --rebuild --steps 100"; do
for pr in "" "--lane-priority 0" "--lane-priority -1"; do
  v="$base $pr"
  tag=$(echo "$v" | tr ' /' '__' | tr -d -)
  timeout -k 10 300 python3 bench.py --config $v --no-cpu-baseline > $OUT/${tag}_$rep.log 2>&1 || { echo "fail $v"; tail -3 $OUT/${tag}_$rep.log; exit 1; }
  echo "$v rep $rep: $(grep -o '"ms_per_step": [0-9.]*' $OUT/${tag}_$rep.log)"
done; done; done
