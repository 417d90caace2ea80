#!/bin/bash
# A/B of option "inst_by_slot" (instance records in TLAS leaf-slot order) on the default C2 bench,
# alternating runs to spread box drift over both arms.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
out=gpurun_out/inst_order_ab.jsonl
: > $out
for rep in 1 2 3; do
  for v in 0 1; do
    timeout -k 10 120 python bench.py --no-cpu-baseline --opt inst_by_slot=$v >> $out || exit $?
  done
done
python - <<'PY'
import json
for l in open("gpurun_out/inst_order_ab.jsonl"):
    d = json.loads(l); c = d["config"]
    print(f'{c["options"]} ms/frame={d["ms_per_step"]:.4f} kernel_ms={d["kernel_ms"]:.4f} frac={d["roofline"]["frac"]:.3f} Mrays/s={d["value"]:.0f}')
PY
