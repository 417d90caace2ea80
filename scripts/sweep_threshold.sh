#!/bin/bash
# Refill-threshold sweep of the overlapped C2 bench, then the N=8 shares with 3 lanes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
out=gpurun_out/sweep.jsonl
: > $out
for t in ${THRESHOLDS:-8 12 16 20 24 32}; do
  timeout -k 10 120 python bench.py --steps 40 --no-cpu-baseline --threshold $t >> $out || exit $?
done
for ((R = 0; R < 8; R++)); do
  timeout -k 10 120 python bench.py --steps 40 --no-cpu-baseline --overlap 3 --shard $R/8 >> $out || exit $?
done
python - <<'PY'
import json
for l in open("gpurun_out/sweep.jsonl"):
    d = json.loads(l); c = d["config"]
    print(f'{c["parallelism"]:28s} lanes={c["overlap_lanes"]} thr={c.get("threshold")} ms/frame={d["ms_per_step"]:.4f} kernel_ms={d["kernel_ms"]:.4f} frac={d["roofline"]["frac"]:.3f} Mrays/s={d["value"]:.0f}')
PY
