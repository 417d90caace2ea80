#!/bin/bash
# rank 0 traces its tiles straight into the frame: multi-GPU tests, A/B vs HEAD (plain C2, share, world-1 comm path)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/dir
mkdir -p $OUT
step() { local name=$1 to=$2; shift 2; echo "=== $name"; timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "rc=$rc"; tail -3 "$OUT/$name.log" | cut -c1-300; [ $rc -eq 0 ] || exit $rc; }
step tests 600 python -u -m pytest tests/test_gpu_multigpu.py tests/test_gpu_parity.py tests/test_gpu_interactive.py -m gpu -x -q --timeout 120 --timeout-method thread
rm -f gpurun_out/ab.jsonl

step ab_comm 900 bash scripts/ab_libs.sh 2 "head=librtamd_head.so new=default" --attach-comm
step ab_comm8 900 bash scripts/ab_libs.sh 1 "head=librtamd_head.so new=default" --attach-comm --overlap 8 --steps 200
step ab_s4 900 bash scripts/ab_libs.sh 1 "head=librtamd_head.so new=default" --shard 4/8 --steps 200
cp gpurun_out/ab.jsonl $OUT/ab.jsonl
exit 0
