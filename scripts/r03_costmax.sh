#!/bin/bash
# cost_max A/B under the auto threshold (whole-wave batches for C2): default line and all-serialised line
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/cm
mkdir -p $OUT
rm -f $OUT/ab.jsonl
for rep in 1 2 3; do
for o in "" "--opt cost_max=1" "--opt split=65535" "--opt cost_max=1 --opt split=65535"; do
  for args in "" "--overlap 1 --clock-warmup 0.3"; do
    timeout -k 10 240 python bench.py --no-cpu-baseline $o $args > $OUT/_b.log 2>&1
    rc=$?; if [ $rc -ne 0 ]; then echo "rc=$rc $o $args"; tail -3 $OUT/_b.log; exit $rc; fi
    grep '^{"metric' $OUT/_b.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'opts': '$o', 'args': '$args', 'ms_per_step': d['ms_per_step'], 'kernel_ms': d['kernel_ms'], 'frac': d['roofline']['frac'], 'lat': d['frame_latency_ms_median']}))" | tee -a $OUT/ab.jsonl
  done
done
done
exit 0
