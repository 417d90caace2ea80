#!/bin/bash
# A/B of option "blas_leaf" (SAH BLAS leaf size, set before the build) on C2 and C3, alternating runs.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
out=gpurun_out/blas_leaf_ab.jsonl
: > $out
for rep in 1 2; do
  for v in 4 2 1; do
    timeout -k 10 120 python bench.py --no-cpu-baseline --pre-opt blas_leaf=$v >> $out || exit $?
  done
done
for v in 4 2; do
  timeout -k 10 200 python bench.py --config C3 --no-cpu-baseline --pre-opt blas_leaf=$v >> $out || exit $?
done
python - <<'PY'
import json
for l in open("gpurun_out/blas_leaf_ab.jsonl"):
    d = json.loads(l); c = d["config"]; w = d["roofline"]["work_per_launch"]
    print(f'{c["workload"][:3]} {c["options"]} ms/frame={d["ms_per_step"]:.4f} kernel_ms={d["kernel_ms"]:.4f} frac={d["roofline"]["frac"]:.3f} Mrays/s={d["value"]:.0f} aabb={w["aabb_tests"]} tri={w["triangle_tests"]}')
PY
