#!/bin/bash
# Round-2 sweeps on one GPU: overlap lanes x reserve, threshold, and the C4 per-rank shares.
# usage: sweep_r02.sh [what]  (what: lanes | thr | c4 | all; outputs gpurun_out/sweep_*.jsonl)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
WHAT=${1:-all}
one() {  # out args...
  local out=$1; shift
  timeout -k 10 240 python bench.py --no-cpu-baseline "$@" > gpurun_out/_one.log 2>&1
  local rc=$?
  if [ $rc -ne 0 ]; then echo "rc=$rc for $*"; tail -3 gpurun_out/_one.log; exit $rc; fi
  tail -1 gpurun_out/_one.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'args': '$*', 'value': d['value'], 'ms_per_step': d['ms_per_step'], 'kernel_ms': d['kernel_ms'], 'kernel_ms_overlapped': d['kernel_ms_overlapped'], 'lat': d['frame_latency_ms_median']}))" | tee -a "gpurun_out/$out"
}
if [[ $WHAT == lanes || $WHAT == all ]]; then
  for rep in 1 2; do for L in 2 3 4; do for rs in 0 8 16; do one sweep_lanes.jsonl --overlap $L --opt reserve=$rs; done; done; done
fi
if [[ $WHAT == thr || $WHAT == all ]]; then
  for t in 24 32 40 48; do one sweep_thr.jsonl --threshold $t ${THR_ARGS:-}; done
fi
if [[ $WHAT == c4 || $WHAT == all ]]; then
  one sweep_c4.jsonl --config C4 ${C4_ARGS:-}
  for r in 0 1 2 3 4 5 6 7; do one sweep_c4.jsonl --config C4 --shard $r/8 ${C4_ARGS:-}; done
fi
exit 0
