#!/bin/bash
# Round-4 final measurement of one library build (everything under gpurun_out/final4/):
#   GPU tests (full-frame parity bars for C2 / C3 / C4 / C5, fake-RCCL worlds), then per config the default
#   (pipelined) bench line, the serialised bench line (--overlap 1), rocprofv3 --kernel-trace --stats of that same
#   serialised command, and the tagged FETCH_SIZE / WRITE_SIZE passes (scripts/pmc_tagged.sh) bench.py prices
#   `traffic` with; the driver's own command last.
# usage: [CONFIGS="C2:sah ..."] [NO_TESTS=1] scripts/r04_final.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${FINAL_OUT:-final4}
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
[ -z "$NO_TESTS" ] && run tests 1100 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread
for spec in ${CONFIGS:-C2:sah C3:sah C4:sah C2:lbvh C5:lbvh:rebuild C5:lbvh}; do
  IFS=: read -r cfg build rb <<< "$spec"
  tag="${cfg}_${build}${rb:+_rebuild}"
  args="--config $cfg --build $build ${rb:+--rebuild}"
  steps=100; [ "$cfg" = C3 ] && steps=40; [ "$cfg" = C5 ] && steps=12
  cpu="--no-cpu-baseline"; [ "$tag" = C2_sah ] && cpu=""
  run "bench_$tag" 600 python3 bench.py $args --steps $steps $cpu
  run "serial_$tag" 600 python3 bench.py $args --overlap 1 --steps $steps --no-cpu-baseline
  run "kstats_$tag" 600 rocprofv3 --kernel-trace --stats -d "$OUT/kstats_$tag" -o run --output-format csv -- \
      python3 bench.py $args --overlap 1 --steps $steps --no-cpu-baseline
  run "pmc_$tag" 900 bash scripts/pmc_tagged.sh "$OUT/pmc_$tag" -- $args
done
run bench_driver 300 python3 bench.py --gpus 1 --steps 20 --warmup 5
run bench_share8 300 python3 bench.py --steps 100 --shard 0/8 --no-cpu-baseline
exit 0
