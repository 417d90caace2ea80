#!/bin/bash
# C5 (per-frame LBVH rebuild) pipeline sweep: lanes, reserved slots, grid share
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/c5s
mkdir -p $OUT
rm -f $OUT/ab.jsonl
for o in "--overlap 3" "--overlap 2" "--overlap 4" "--overlap 3 --opt reserve=64" "--overlap 3 --opt reserve=128" "--overlap 3 --opt grid_pct=40" "--overlap 2 --opt reserve=64"; do
  timeout -k 10 300 python bench.py --config C5 --build lbvh --rebuild --steps 12 --no-cpu-baseline $o > $OUT/_b.log 2>&1
  rc=$?; if [ $rc -ne 0 ]; then echo "rc=$rc $o"; tail -3 $OUT/_b.log; exit $rc; fi
  grep '^{"metric' $OUT/_b.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'opts': '$o', 'ms_per_step': d['ms_per_step'], 'kernel_ms': d['kernel_ms'], 'kernel_ms_overlapped': d['kernel_ms_overlapped'], 'lat': d['frame_latency_ms_median']}))" | tee -a $OUT/ab.jsonl
done
exit 0
