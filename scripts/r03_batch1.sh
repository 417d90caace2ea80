#!/bin/bash
# write-size calibration (scripts/write_cal.hip), C2-LBVH / C2-SAH kernel traces, 1/8 shares of C2 and C4
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/b1
mkdir -p $OUT
export TMPDIR=/tmp
step() { local name=$1 to=$2; shift 2; echo "=== $name"; timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "rc=$rc"; tail -2 "$OUT/$name.log" | cut -c1-300; [ $rc -eq 0 ] || exit $rc; }
step wcal 120 rocprofv3 --pmc WRITE_SIZE -d $OUT/wcal -o run --output-format csv -- ./scripts/write_cal
step ktrace_lbvh 300 rocprofv3 --kernel-trace -d $OUT/kt_lbvh -o run --output-format csv -- python3 bench.py --build lbvh --steps 40 --warmup 5 --no-cpu-baseline --clock-warmup 0
step ktrace_sah 300 rocprofv3 --kernel-trace -d $OUT/kt_sah -o run --output-format csv -- python3 bench.py --steps 40 --warmup 5 --no-cpu-baseline --clock-warmup 0
for cfg in C2 C4; do
  for r in 0 1 2 3 4 5 6 7; do
    step share_${cfg}_$r 120 python3 bench.py --config $cfg --shard $r/8 --steps 200 --no-cpu-baseline
    tail -1 $OUT/share_${cfg}_$r.log >> $OUT/shares.jsonl
  done
done
