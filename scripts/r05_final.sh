#!/bin/bash
# Round-5 final measurement of one library build (everything under gpurun_out/final5/):
#   GPU tests, then per config the default (pipelined) bench line, the serialised bench line (--overlap 1),
#   rocprofv3 --kernel-trace --stats of that same serialised command, and the tagged PMC passes
#   (scripts/pmc_tagged.sh: FETCH_SIZE / WRITE_SIZE, plus for C2 / C3 / C5 the deep set — occupancy, VALU lane use,
#   L2 hit, L1 latency) bench.py prices `traffic` with; the driver's own command last.  Raw counter / trace CSVs are
#   deleted once summarised (gpurun_out merges back only under 64 MiB).
# usage: [CONFIGS="C2:sah ..."] [NO_TESTS=1] [NO_DRIVER=1] scripts/r05_final.sh   (two calls: each under 20 min)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${FINAL_OUT:-final5}
mkdir -p $OUT
export TMPDIR=/tmp
run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "=== $name"
  timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "rc=$rc"; tail -1 "$OUT/$name.log" | cut -c1-240
  if [ $rc -ne 0 ]; then tail -8 "$OUT/$name.log"; exit $rc; fi
}
[ -z "$NO_TESTS" ] && run tests 600 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread
for spec in ${CONFIGS:-C2:sah C3:sah C4:sah C2:lbvh C5:lbvh:rebuild C5:lbvh}; do
  IFS=: read -r cfg build rb <<< "$spec"
  tag="${cfg}_${build}${rb:+_rebuild}"
  args="--config $cfg --build $build ${rb:+--rebuild}"
  steps=100; [ "$cfg" = C3 ] && steps=40; [ "$cfg" = C5 ] && steps=12
  cpu="--no-cpu-baseline"; [ "$tag" = C2_sah ] && cpu=""
  deep=""; case "$tag" in C2_sah|C3_sah|C5_lbvh) deep=deep;; esac
  run "bench_$tag" 600 python3 bench.py $args --steps $steps $cpu
  run "serial_$tag" 600 python3 bench.py $args --overlap 1 --steps $steps --no-cpu-baseline
  run "kstats_$tag" 600 rocprofv3 --kernel-trace --stats -d "$OUT/kstats_$tag" -o run --output-format csv -- \
      python3 bench.py $args --overlap 1 --steps $steps --no-cpu-baseline
  find "$OUT/kstats_$tag" -name '*kernel_trace.csv' -delete
  PMC_SET=$deep PMC_STEPS=$([ "$cfg" = C5 ] && echo 3 || echo 5) run "pmc_$tag" 900 bash scripts/pmc_tagged.sh "$OUT/pmc_$tag" -- $args
  rm -rf "$OUT"/pmc_$tag/pass*/
done
if [ -z "$NO_DRIVER" ]; then
  run bench_driver 300 python3 bench.py --gpus 1 --steps 20 --warmup 5
  run bench_share8 300 python3 bench.py --steps 100 --shard 0/8 --no-cpu-baseline
fi
exit 0
