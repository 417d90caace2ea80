#!/bin/bash
# Study (2): high-priority overlap lanes on the other workloads: C5 static, C3, 1/8 shares, the world-1 comm path.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/prio2; mkdir -p $OUT
for rep in 1 2; do
for base in "C5 --build lbvh --steps 12" "C3 --steps 40" "C2 --shard 0/8 --steps 200" "C4 --shard 2/8 --steps 200" "C2 --attach-comm --steps 100" "C2 --build lbvh --rebuild --steps 100"; do
for pr in "" "--lane-priority -1"; do
  v="$base $pr"
  tag=$(echo "$v" | tr ' /' '__' | tr -d -)
  timeout -k 10 300 python3 bench.py --config $v --no-cpu-baseline > $OUT/${tag}_$rep.log 2>&1 || { echo "fail $v"; tail -3 $OUT/${tag}_$rep.log; exit 1; }
  echo "$v rep $rep: $(grep -o '"ms_per_step": [0-9.]*' $OUT/${tag}_$rep.log)"
done; done; done
