#!/bin/bash
# HIP API + kernel traces of the one-GPU 1/8 share (8 lanes): when the host enqueues each frame vs when the GPU runs it
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/st
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --hip-trace --kernel-trace -d $OUT/ht_share -o run --output-format csv -- \
    python3 bench.py --shard 4/8 --steps 200 --no-cpu-baseline --clock-warmup 0.2 ${EXTRA:-} > $OUT/ht_share.log 2>&1
rc=$?; echo "rc=$rc"; tail -1 $OUT/ht_share.log | cut -c1-200; exit $rc
