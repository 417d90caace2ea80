#!/bin/bash
# world-1 comm path: hardware queues per process vs lanes (the N > 1 bench sets 12)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/cq
mkdir -p $OUT
rm -f $OUT/ab.jsonl
for q in 12 16 24; do
  for L in 3 8; do
    RTAMD_HWQ=$q timeout -k 10 240 python bench.py --attach-comm --overlap $L --no-cpu-baseline --steps 200 > $OUT/_b.log 2>&1
    rc=$?; if [ $rc -ne 0 ]; then echo "rc=$rc q=$q L=$L"; tail -3 $OUT/_b.log; exit $rc; fi
    grep '^{"metric' $OUT/_b.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'hwq': $q, 'lanes': $L, 'ms_per_step': d['ms_per_step'], 'kernel_ms_overlapped': d['kernel_ms_overlapped']}))" | tee -a $OUT/ab.jsonl
    RTAMD_HWQ=$q timeout -k 10 240 python bench.py --shard 4/8 --overlap $L --no-cpu-baseline --steps 200 > $OUT/_b.log 2>&1
    grep '^{"metric' $OUT/_b.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'hwq': $q, 'lanes': $L, 'shard': '4/8', 'ms_per_step': d['ms_per_step'], 'kernel_ms_overlapped': d['kernel_ms_overlapped']}))" | tee -a $OUT/ab.jsonl
  done
done
exit 0
