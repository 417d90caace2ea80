#!/bin/bash
# full-frame C2 pipeline: overlap lanes x hardware queues
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/lq
mkdir -p $OUT
rm -f $OUT/ab.jsonl
for rep in 1 2; do
for q in 4 8 16; do
  for L in 3 4 6; do
    RTAMD_HWQ=$q timeout -k 10 240 python bench.py --no-cpu-baseline --overlap $L > $OUT/_b.log 2>&1
    rc=$?; if [ $rc -ne 0 ]; then echo "rc=$rc q=$q L=$L"; tail -3 $OUT/_b.log; exit $rc; fi
    grep '^{"metric' $OUT/_b.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'hwq': $q, 'lanes': $L, 'ms_per_step': d['ms_per_step'], 'value': d['value'], 'kernel_ms_overlapped': d['kernel_ms_overlapped']}))" | tee -a $OUT/ab.jsonl
  done
done
done
exit 0
