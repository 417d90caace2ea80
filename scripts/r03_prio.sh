#!/bin/bash
# Study: overlap lanes on high-priority HIP streams (the library's scene stream, which runs the per-frame
# BLAS rebuild, stays at normal priority).  One bench line per variant into gpurun_out/prio/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/prio; mkdir -p $OUT
python3 -c "import torch; print('priority_range', torch.cuda.Stream.priority_range())"
for rep in 1 2; do
for v in "C5 --rebuild" "C5 --rebuild --lane-priority -1" "C2" "C2 --lane-priority -1"; do
  set -- $v
  tag=$(echo "$v" | tr ' ' '_' | tr -d -)
  timeout -k 10 300 python3 bench.py --config $v $( [ $1 = C5 ] && echo "--build lbvh --steps 12" || echo "--steps 100") \
      --no-cpu-baseline > $OUT/${tag}_$rep.log 2>&1 || { echo "fail $v"; tail -3 $OUT/${tag}_$rep.log; exit 1; }
  echo "$v rep $rep: $(grep -o '"ms_per_step": [0-9.]*' $OUT/${tag}_$rep.log)"
done; done
