#!/bin/bash
# self_reset / copy_sdma: byte-identity tests, then shares and the full frame A/B (one library, options)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/sr
mkdir -p $OUT
step() { local name=$1 to=$2; shift 2; echo "=== $name"; timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "rc=$rc"; tail -3 "$OUT/$name.log" | cut -c1-300; [ $rc -eq 0 ] || exit $rc; }
step tests 600 python -u -m pytest tests/test_gpu_parity.py -k "claim_options or reorder_period" -m gpu -x -q --timeout 120 --timeout-method thread
rm -f $OUT/ab.jsonl
for rep in 1 2; do
for o in "" "--opt self_reset=1"; do
  for args in "--shard 4/8 --steps 200" "--config C4 --shard 3/8 --steps 200" ""; do
    timeout -k 10 240 python bench.py --no-cpu-baseline $o $args > $OUT/_b.log 2>&1
    rc=$?; if [ $rc -ne 0 ]; then echo "rc=$rc $o $args"; tail -3 $OUT/_b.log; exit $rc; fi
    grep '^{"metric' $OUT/_b.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'opts': '$o', 'args': '$args', 'ms_per_step': d['ms_per_step'], 'kernel_ms': d['kernel_ms'], 'kernel_ms_overlapped': d['kernel_ms_overlapped'], 'lat': d['frame_latency_ms_median']}))" | tee -a $OUT/ab.jsonl
  done
done
done
exit 0
