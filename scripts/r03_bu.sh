#!/bin/bash
# chunked bottom-up (LBVH > 2048 items): LBVH tests, C5 / C2-LBVH A/B vs HEAD, C5 kernel stats
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/bu
mkdir -p $OUT
export TMPDIR=/tmp
step() { local name=$1 to=$2; shift 2; echo "=== $name"; timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "rc=$rc"; tail -3 "$OUT/$name.log" | cut -c1-300; [ $rc -eq 0 ] || exit $rc; }
step tests 900 python -u -m pytest tests/test_gpu_lbvh.py tests/test_gpu_configs.py tests/test_gpu_group.py -m gpu -x -q --timeout 300 --timeout-method thread
rm -f gpurun_out/ab.jsonl
step ab_c5 900 bash scripts/ab_libs.sh 2 "head=librtamd_head.so new=default" --config C5 --build lbvh --rebuild --steps 12
step ab_c2l 600 bash scripts/ab_libs.sh 2 "head=librtamd_head.so new=default" --build lbvh --rebuild

cp gpurun_out/ab.jsonl $OUT/ab.jsonl
step kst 600 rocprofv3 --kernel-trace --stats -d $OUT/kst -o run --output-format csv -- python3 bench.py --config C5 --build lbvh --rebuild --steps 12 --no-cpu-baseline
exit 0
