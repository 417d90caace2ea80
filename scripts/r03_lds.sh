#!/bin/bash
# A/B: HEAD vs the 16 B page helpers (default) vs smaller LDS stack windows with a larger LDS scene region
# (w12: 12 entries + 27 KB, w8: 8 entries + 35 KB); WRITE_SIZE of the grid kernel (one store per 8x8 unit)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/lds
mkdir -p $OUT
export TMPDIR=/tmp
step() { local name=$1 to=$2; shift 2; echo "=== $name"; timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "rc=$rc"; tail -3 "$OUT/$name.log" | cut -c1-300; [ $rc -eq 0 ] || exit $rc; }
rm -f gpurun_out/ab.jsonl
V=${V:-"head=librtamd_head.so new=default w12=librtamd_w12.so w8=librtamd_w8.so"}
step ab_c2 900 bash scripts/ab_libs.sh 3 "$V"
step ab_c3 600 bash scripts/ab_libs.sh 1 "$V" --config C3 --steps 40
step ab_s4 600 bash scripts/ab_libs.sh 1 "$V" --shard 4/8 --steps 200
cp gpurun_out/ab.jsonl $OUT/ab.jsonl
step ws_grid 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/ws_grid -o run --output-format csv -- \
    python3 bench.py --kernel 0 --steps 5 --warmup 2 --overlap 1 --no-cpu-baseline --clock-warmup 0
step ws_nt 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/ws_nt -o run --output-format csv -- \
    python3 bench.py --opt nt_store=1 --steps 5 --warmup 2 --overlap 1 --no-cpu-baseline --clock-warmup 0
exit 0
