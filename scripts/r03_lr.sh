#!/bin/bash
# quad steps read one ray register set (lr, the world ray restored after an instance) vs HEAD
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/lr
mkdir -p $OUT
step() { local name=$1 to=$2; shift 2; echo "=== $name"; timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "rc=$rc"; tail -3 "$OUT/$name.log" | cut -c1-300; [ $rc -eq 0 ] || exit $rc; }
step tests 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_group.py tests/test_gpu_configs.py -m gpu -x -q --timeout 120 --timeout-method thread
rm -f gpurun_out/ab.jsonl
step ab_c2 900 bash scripts/ab_libs.sh 3 "head=librtamd_head.so new=default"
step ab_c2s 900 bash scripts/ab_libs.sh 2 "head=librtamd_head.so new=default" --overlap 1 --clock-warmup 0.3
step ab_c3 600 bash scripts/ab_libs.sh 1 "head=librtamd_head.so new=default" --config C3 --steps 40
cp gpurun_out/ab.jsonl $OUT/ab.jsonl
exit 0
