#!/bin/bash
# Round-6 session: the GPU builder's tests, then the rebuild alone and C5 with the rebuild, 2048- against 1024-item
# bottom-up chunks (librtamd_chunk1k.so), interleaved.
cd ${GRAFT_REPO_ROOT:-$(dirname "$0")/..}
export TMPDIR=/tmp
OUT=gpurun_out/${S_OUT:-r06s11}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_lbvh.py tests/test_gpu_parity_full.py -k "lbvh or C5" -q -rf --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $OUT/tests.log; [ $rc -ne 0 ] && exit $rc
for rep in 1 2 3; do
  for v in default chunk1k; do
    lib=""; [ $v != default ] && lib=$PWD/real-time-gpu-ray-tracer_amd/lib/librtamd_$v.so
    RTAMD_LIB=$lib timeout -k 10 300 python3 scripts/rebuild_alone.py --updates 30 > $OUT/alone_${v}_$rep.log 2>&1 || exit 1
    echo "alone $v $(tail -1 $OUT/alone_${v}_$rep.log)"
  done
done
OPT=lib VALS="default chunk1k" REPS=2 CASES="c5rb|--config C5 --build lbvh --rebuild --steps 12;c5s8|--config C5 --build lbvh --rebuild --shard 0/8 --steps 24" bash scripts/ab.sh ${S_OUT:-r06s11}/ab
