#!/bin/bash
# One-GPU study of option "overlap": N=1 frame throughput, and each rank's share of an N-rank split
# (bench.py --shard R/N) for several lane counts (1 = frames serialised).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
out=gpurun_out/overlap_study.jsonl
: > $out
for L in ${LANES:-1 2 3 4}; do
  timeout -k 10 120 python bench.py --steps ${STEPS:-40} --no-cpu-baseline --overlap $L >> $out || exit $?
done
for N in ${NS:-8}; do
  for L in ${SHARD_LANES:-1 2 4}; do
    for ((R = 0; R < N; R++)); do
      timeout -k 10 120 python bench.py --steps ${STEPS:-40} --no-cpu-baseline --overlap $L --shard $R/$N >> $out || exit $?
    done
  done
done
python - <<'PY'
import json
for l in open("gpurun_out/overlap_study.jsonl"):
    d = json.loads(l)
    c = d["config"]
    print(f'{c["parallelism"]:32s} lanes={c["overlap_lanes"]} ms/frame={d["ms_per_step"]:.4f} kernel_ms={d["kernel_ms"]:.4f} Mrays/s={d["value"]:.0f}')
PY
