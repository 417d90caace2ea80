#!/bin/bash
# workgroup claim buffer A/B (RT_WG_CLAIM 4 default vs 1 = per-wave claims, 2) + parity tests
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/wg
mkdir -p $OUT
step() { local name=$1 to=$2; shift 2; echo "=== $name"; timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "rc=$rc"; tail -3 "$OUT/$name.log" | cut -c1-300; [ $rc -eq 0 ] || exit $rc; }
step tests 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_multigpu.py -m gpu -x -q --timeout 120 --timeout-method thread
rm -f gpurun_out/ab.jsonl
V=${V:-"wg1=librtamd_wg1.so wg4=default wg2=librtamd_wg2.so"}
step ab_c2 900 bash scripts/ab_libs.sh 3 "$V"
step ab_c3 600 bash scripts/ab_libs.sh 1 "$V" --config C3 --steps 40
step ab_s4 600 bash scripts/ab_libs.sh 1 "$V" --shard 4/8 --steps 200
step ab_c4 600 bash scripts/ab_libs.sh 1 "$V" --config C4
cp gpurun_out/ab.jsonl $OUT/ab.jsonl
exit 0
