#!/bin/bash
# r05 session 13: full GPU suite on the new defaults; share lanes' priority at 24 queues (bench's N > 1 setting)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05s13; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -4 $O/gpu_tests.log; [ $rc -ne 0 ] && exit $rc
one() {   # name hwq args...
  local name=$1 q=$2; shift 2
  RTAMD_HWQ=$q timeout -k 10 300 python3 bench.py "$@" --no-cpu-baseline > $O/$name.log 2>&1 || { echo "fail $name"; tail -5 $O/$name.log; exit 1; }
  python3 - $O/$name.log $name <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().split("\n")[-1])
print(f"{sys.argv[2]:18s} hwq {d['config']['hw_queues']:>2d} lanes {d['config']['overlap_lanes']} ms/frame {d['ms_per_step']:.4f} lat {d['frame_latency_ms_median']:.4f}", flush=True)
PY
}
for rep in 1 2; do
  one share_p1_q24_$rep 24 --steps 100 --shard 0/8
  one share_p0_q24_$rep 24 --steps 100 --shard 0/8 --opt lane_priority=0
  one share_p0_q12_$rep 12 --steps 100 --shard 0/8 --opt lane_priority=0
  one share4_p1_q24_$rep 24 --config C4 --steps 100 --shard 2/8
  one share4_p0_q24_$rep 24 --config C4 --steps 100 --shard 2/8 --opt lane_priority=0
done
