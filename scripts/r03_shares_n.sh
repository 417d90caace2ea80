#!/bin/bash
# lanes per rank for N = 2 and 4 (one-GPU share study: rank 0's 1/N share), 3 / 4 / 6 / 8 lanes
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/sn
mkdir -p $OUT
rm -f $OUT/ab.jsonl
for rep in 1 2; do
for n in 2 4; do
  for L in 3 4 6 8; do
    timeout -k 10 240 python bench.py --no-cpu-baseline --shard 0/$n --overlap $L --steps 200 > $OUT/_b.log 2>&1
    rc=$?; if [ $rc -ne 0 ]; then echo "rc=$rc n=$n L=$L"; tail -3 $OUT/_b.log; exit $rc; fi
    grep '^{"metric' $OUT/_b.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'n': $n, 'lanes': $L, 'ms_per_step': d['ms_per_step'], 'kernel_ms_overlapped': d['kernel_ms_overlapped'], 'lat': d['frame_latency_ms_median']}))" | tee -a $OUT/ab.jsonl
  done
done
done
exit 0
