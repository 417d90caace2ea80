#!/bin/bash
# Kernel traces of the one-GPU 1/8 share (8 lanes): what sits between a lane's trace launches
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/st
mkdir -p $OUT
export TMPDIR=/tmp
step() { local name=$1 to=$2; shift 2; echo "=== $name"; timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "rc=$rc"; tail -2 "$OUT/$name.log" | cut -c1-300; [ $rc -eq 0 ] || exit $rc; }
step kt_share 300 rocprofv3 --kernel-trace -d $OUT/kt_share -o run --output-format csv -- \
    python3 bench.py --shard 4/8 --steps 200 --no-cpu-baseline ${EXTRA:-}
step kt_share_skip 300 rocprofv3 --kernel-trace -d $OUT/kt_share_skip -o run --output-format csv -- \
    python3 bench.py --shard 4/8 --steps 200 --no-cpu-baseline --skip-update ${EXTRA:-}
exit 0
