#!/bin/bash
# staging depth A/B (option "stage_depth"): 1/8 shares (8 lanes) and the full frame (3 lanes)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/stage
mkdir -p $OUT
rm -f $OUT/ab.jsonl
for rep in 1 2; do
for d in ${DEPTHS:-16 32 64}; do
  for args in "--shard 4/8 --steps 200" "--shard 1/8 --steps 200" "--config C4 --shard 3/8 --steps 200" ""; do
    timeout -k 10 240 python bench.py --no-cpu-baseline --opt stage_depth=$d $args > $OUT/_b.log 2>&1
    rc=$?; if [ $rc -ne 0 ]; then echo "rc=$rc d=$d $args"; tail -3 $OUT/_b.log; exit $rc; fi
    grep '^{"metric' $OUT/_b.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'depth': $d, 'args': '$args', 'ms_per_step': d['ms_per_step'], 'kernel_ms_overlapped': d['kernel_ms_overlapped'], 'call_mean': d['host_call_ms_mean'], 'wait_mean': d['host_update_wait_ms_mean'], 'busy': d['host_busy_ms_median']}))" | tee -a $OUT/ab.jsonl
  done
done
done
exit 0
