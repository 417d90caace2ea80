#!/bin/bash
# Heavy-unit split levels ("split" = k_half | k_quarter << 8) and bands for a rank's 1/8 share and the full frame.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
out=gpurun_out/split_study.jsonl
: > $out
for o in "split=0x0C0A" "split=0x0806" "split=0x0604" "split=0x0402" "queue_parts=4" "queue_parts=1"; do
  for sh in 3/8 4/8 5/8; do
    timeout -k 10 120 python bench.py --steps 40 --no-cpu-baseline --overlap 3 --shard $sh --opt $o >> $out || exit $?
  done
  timeout -k 10 120 python bench.py --steps 40 --no-cpu-baseline --opt $o >> $out || exit $?
done
python - <<'PY'
import json
for l in open("gpurun_out/split_study.jsonl"):
    d = json.loads(l); c = d["config"]
    print(f'{c["parallelism"]:28s} {c["options"]} lanes={c["overlap_lanes"]} ms/frame={d["ms_per_step"]:.4f} kernel_ms={d["kernel_ms"]:.4f} frac={d["roofline"]["frac"]:.3f}')
PY
