#!/bin/bash
# Per config: the serialised bench line (--overlap 1), rocprofv3 --kernel-trace --stats of the same command,
# and tagged FETCH_SIZE / WRITE_SIZE passes (scripts/pmc_tagged.sh).  Outputs under gpurun_out/meas/.
# usage: CONFIGS="C2:sah C3:sah C4:sah C5:lbvh:rebuild" scripts/r03_measure.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/meas
mkdir -p $OUT
export TMPDIR=/tmp
run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "=== $name: $*"
  timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -2 "$OUT/$name.log" | cut -c1-400
  if [ $rc -ne 0 ]; then exit $rc; fi
}
for spec in ${CONFIGS:-C2:sah C3:sah C4:sah C5:lbvh:rebuild}; do
  IFS=: read -r cfg build rb <<< "$spec"
  args="--config $cfg --build $build ${rb:+--rebuild}"
  steps=100; [ "$cfg" = C3 ] && steps=40; [ "$cfg" = C5 ] && steps=12
  run "bench_$cfg" 600 python3 bench.py $args --overlap 1 --steps $steps --no-cpu-baseline
  run "kstats_$cfg" 600 rocprofv3 --kernel-trace --stats -d "$OUT/kstats_$cfg" -o run --output-format csv -- \
      python3 bench.py $args --overlap 1 --steps $steps --no-cpu-baseline
  run "pmc_$cfg" 900 bash scripts/pmc_tagged.sh "$OUT/pmc_$cfg" -- $args
done
exit 0
