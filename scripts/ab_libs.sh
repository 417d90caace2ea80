#!/bin/bash
# Alternating A/B of library builds on one GPU: scripts/ab_libs.sh REPS "tag=libfile ..." [bench args]
# (libfile relative to real-time-gpu-ray-tracer_amd/lib; "default" = librtamd.so); one JSON line per run
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
REPS=$1; VARIANTS=$2; shift 2
for rep in $(seq 1 "$REPS"); do
  for v in $VARIANTS; do
    tag=${v%%=*}; lib=${v#*=}
    [ "$lib" = default ] && lib=librtamd.so
    RTAMD_LIB=$PWD/real-time-gpu-ray-tracer_amd/lib/$lib timeout -k 10 240 python bench.py --no-cpu-baseline "$@" > gpurun_out/_ab.log 2>&1
    rc=$?
    if [ $rc -ne 0 ]; then echo "rc=$rc for $tag"; tail -3 gpurun_out/_ab.log; exit $rc; fi
    tail -1 gpurun_out/_ab.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'tag': '$tag', 'args': '$*', 'value': d['value'], 'ms_per_step': d['ms_per_step'], 'kernel_ms': d['kernel_ms'], 'kernel_ms_overlapped': d['kernel_ms_overlapped'], 'lat': d['frame_latency_ms_median'], 'frac': d['roofline']['frac']}))" | tee -a gpurun_out/ab.jsonl
  done
done
