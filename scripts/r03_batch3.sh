#!/bin/bash
# spill fixes: parity tests, A/B vs the HEAD kernel (C2 x3, C3 x1), WRITE_SIZE pass
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/b3
mkdir -p $OUT
export TMPDIR=/tmp
step() { local name=$1 to=$2; shift 2; echo "=== $name"; timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "rc=$rc"; tail -2 "$OUT/$name.log" | cut -c1-400; [ $rc -eq 0 ] || exit $rc; }
step parity 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -q --timeout 120 --timeout-method thread
rm -f gpurun_out/ab.jsonl
step ab_c2 900 bash scripts/ab_libs.sh 3 "head=librtamd_head.so new=default"
step ab_c3 600 bash scripts/ab_libs.sh 1 "head=librtamd_head.so new=default" --config C3 --steps 40
cp gpurun_out/ab.jsonl $OUT/ab.jsonl
step pmc_ws 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_ws -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --overlap 1 --no-cpu-baseline --clock-warmup 0
