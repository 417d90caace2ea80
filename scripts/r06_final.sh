#!/bin/bash
# Round-6 final measurement of one library build (everything under gpurun_out/final6/), in two calls:
#   PART=1: the GPU test suite, the full-frame parity report (-s: outlier counts), then C2 / C3 / C4;
#   PART=2: C2 on GPU trees, C5 (trees built once, and rebuilt every frame: its "rebuild" roofline block), the
#           driver's own command, the 1/8 shares (C2, C5 with the rebuild).
# Per config: the default (pipelined) bench line, the serialised line (--overlap 1), rocprofv3 --kernel-trace --stats
# of that serialised command, and the tagged PMC passes (scripts/pmc_tagged.sh: FETCH_SIZE / WRITE_SIZE, plus for C2 /
# C3 / C5 the deep set) that bench.py prices `traffic` with.  Raw counter / trace CSVs are deleted once summarised.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${FINAL_OUT:-final6}
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
config() {  # spec = cfg:build[:rebuild]
  IFS=: read -r cfg build rb <<< "$1"
  tag="${cfg}_${build}${rb:+_rebuild}"
  args="--config $cfg --build $build ${rb:+--rebuild}"
  steps=100; [ "$cfg" = C3 ] && steps=40; [ "$cfg" = C5 ] && steps=12
  cpu="--no-cpu-baseline"; [ "$tag" = C2_sah ] && cpu=""
  deep=""; case "$tag" in C2_sah|C3_sah|C5_lbvh) deep=deep;; esac
  run "bench_$tag" 600 python3 bench.py $args --steps $steps $cpu
  run "serial_$tag" 600 python3 bench.py $args --overlap 1 --steps $steps --no-cpu-baseline --no-rebuild-roofline
  run "kstats_$tag" 600 rocprofv3 --kernel-trace --stats -d "$OUT/kstats_$tag" -o run --output-format csv -- \
      python3 bench.py $args --overlap 1 --steps $steps --no-cpu-baseline --no-rebuild-roofline
  find "$OUT/kstats_$tag" -name '*kernel_trace.csv' -delete
  PMC_SET=$deep PMC_STEPS=$([ "$cfg" = C5 ] && echo 3 || echo 5) run "pmc_$tag" 900 bash scripts/pmc_tagged.sh "$OUT/pmc_$tag" -- $args
  rm -rf "$OUT"/pmc_$tag/pass*/
}
if [ "${PART:-1}" = 1 ]; then
  run tests 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread
  run parity_full 900 python -u -m pytest tests/test_gpu_parity_full.py -v -s --timeout 600 --timeout-method thread
  for spec in ${CONFIGS:-C2:sah C3:sah C4:sah}; do config $spec; done
else
  for spec in ${CONFIGS:-C2:lbvh C5:lbvh:rebuild C5:lbvh}; do config $spec; done
  run bench_driver 300 python3 bench.py --gpus 1 --steps 20 --warmup 5
  run bench_share8 300 python3 bench.py --steps 100 --shard 0/8 --no-cpu-baseline
  run bench_share8_c5_rebuild 300 python3 bench.py --config C5 --build lbvh --rebuild --shard 0/8 --steps 24 --no-cpu-baseline
fi
exit 0
