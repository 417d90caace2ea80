#!/bin/bash
# LBVH scenes with and without instance groups (option "group"): C2-LBVH, C5 (per-frame rebuild)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/lbvh
mkdir -p $OUT
run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "=== $name: $*"
  timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -1 "$OUT/$name.log" | python3 -c "import json,sys
try:
    d=json.loads(sys.stdin.read()); r=d['roofline']; w=r['work_per_launch']
    print(json.dumps({'value': d['value'], 'ms_per_step': d['ms_per_step'], 'kernel_ms': d['kernel_ms'], 'lat': d['frame_latency_ms_median'], 'frac': r['frac'], 'inst_per_ray': round(w['instance_visits']/w['rays'],3), 'aabb_per_ray': round(w['aabb_tests']/w['rays'],2), 'tri_per_ray': round(w['triangle_tests']/w['rays'],2)}))
except Exception as e: print('unparsed', e)"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
}
run c2_sah 300 python bench.py --no-cpu-baseline
run c2_lbvh_group 300 python bench.py --build lbvh --no-cpu-baseline
run c2_lbvh_nogroup 300 python bench.py --build lbvh --pre-opt group=0 --no-cpu-baseline
run c5_group 600 python bench.py --config C5 --build lbvh --rebuild --steps 12 --warmup 3 --no-cpu-baseline
run c5_nogroup 600 python bench.py --config C5 --build lbvh --rebuild --steps 12 --warmup 3 --pre-opt group=0 --no-cpu-baseline
exit 0
