#!/bin/bash
# Extra bench lines (non-default configs) + a rocprofv3 kernel-stats pass of the C5 GPU-rebuild run.
# usage: bench_configs.sh [tag]   (outputs under gpurun_out/)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-cfg}
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "=== $name: $*"
  timeout -k 10 "$to" "$@" > "gpurun_out/${TAG}_$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -3 "gpurun_out/${TAG}_$name.log"
  if [ $rc -ne 0 ]; then exit $rc; fi
}
step c2_lbvh 300 python bench.py --build lbvh --no-cpu-baseline
step c3_sah 300 python bench.py --config C3 --no-cpu-baseline
step c5_lbvh_rebuild 600 python bench.py --config C5 --build lbvh --rebuild --steps 5 --warmup 2 --no-cpu-baseline
step c5_prof_skip 600 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_c5prof -o run --output-format csv -- python3 bench.py --config C5 --build lbvh --rebuild --steps 5 --warmup 2 --no-cpu-baseline
exit 0
