#!/bin/bash
# One-GPU study of the N-rank screen-tile size: each rank's share (bench.py --shard R/N --tile T).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
out=gpurun_out/tile_study.jsonl
: > $out
for T in ${TILES:-64 32 16}; do
  for N in ${NS:-8 4}; do
    for ((R = 0; R < N; R++)); do
      timeout -k 10 120 python bench.py --steps ${STEPS:-40} --no-cpu-baseline --tile $T --shard $R/$N >> $out || exit $?
    done
  done
done
python - <<'PY'
import json, collections
rows = collections.defaultdict(list)
for l in open("gpurun_out/tile_study.jsonl"):
    d = json.loads(l)
    c = d["config"]
    rows[(c["tile"], c["parallelism"].split()[-2].split("/")[1])].append((d["ms_per_step"], d["kernel_ms"]))
for (t, n), v in rows.items():
    ms = [a for a, _ in v]
    print(f"tile {t} N={n}: slowest {max(ms):.4f} ms/frame, mean {sum(ms)/len(ms):.4f}, fastest {min(ms):.4f}; kernel max {max(k for _, k in v):.4f}")
PY
