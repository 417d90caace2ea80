#!/bin/bash
# Round-4 session 4: where the time goes at the new default (IEEE FAST kernel): launch schedule of the driver's
# 20-step window vs 100 steps, per-wave timelines (diagnostic build) of a whole C2 frame and a synchronous 1/8
# share, the deep PMC set for C2 / C3 / C5 (one counter group per rocprofv3 run), kernel stats of the serialised C2.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r04s4
mkdir -p $OUT
export TMPDIR=/tmp
run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "=== $name"
  timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "rc=$rc"; tail -2 "$OUT/$name.log" | cut -c1-400
  if [ $rc -ne 0 ]; then tail -30 "$OUT/$name.log"; exit $rc; fi
}
run lt20 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --launch-times $OUT/lt20.npy
run lt100 300 python3 bench.py --steps 100 --no-cpu-baseline --launch-times $OUT/lt100.npy
DIAG=$PWD/real-time-gpu-ray-tracer_amd/lib/librtamd_diag.so
RTAMD_LIB=$DIAG run tl_c2 300 python3 scripts/timeline.py --parts 8 --threshold 0 --out $OUT/tl_c2.npz
RTAMD_LIB=$DIAG run tl_c2_share 300 python3 scripts/timeline.py --parts 8 --threshold 0 --shard 0/8 --out $OUT/tl_c2_share.npz
run kstats_c2 300 rocprofv3 --kernel-trace --stats -d $OUT/kstats_c2 -o run --output-format csv -- \
    python3 bench.py --overlap 1 --steps 100 --no-cpu-baseline
for spec in C2:sah C3:sah C5:lbvh; do
  IFS=: read -r cfg build <<< "$spec"
  run pmc_$cfg 1200 bash scripts/pmc_passes.sh $OUT/pmc_$cfg "render_persistent_kernel<false" -- \
      python3 bench.py --config $cfg --build $build --steps 4 --warmup 2 --overlap 1 --no-cpu-baseline --clock-warmup 0.2
done
exit 0
