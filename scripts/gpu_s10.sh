#!/bin/bash
# Round-6 session: the pruned library's bench lines (C2 driver command, C3, C5 static, C5 with the rebuild and its
# "rebuild" roofline block, the C5 1/8 share with the rebuild), then a rocprofv3 kernel trace of the rebuild alone.
cd ${GRAFT_REPO_ROOT:-$(dirname "$0")/..}
export TMPDIR=/tmp
OUT=gpurun_out/${S_OUT:-r06s10}; mkdir -p $OUT
run() { local name=$1 to=$2; shift 2; timeout -k 10 $to "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; \
        tail -1 $OUT/$name.log | cut -c1-400; [ $rc -ne 0 ] && { tail -5 $OUT/$name.log; exit $rc; }; return 0; }
run c2_driver 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline
run c3 300 python3 bench.py --config C3 --steps 40 --no-cpu-baseline
run c5 300 python3 bench.py --config C5 --build lbvh --steps 12 --no-cpu-baseline
run c5rb 300 python3 bench.py --config C5 --build lbvh --rebuild --steps 12 --no-cpu-baseline
run c5rb_s8 300 python3 bench.py --config C5 --build lbvh --rebuild --shard 0/8 --steps 24 --no-cpu-baseline
run rb_kstats 300 rocprofv3 --kernel-trace --stats -d $OUT/rb_kstats -o run --output-format csv -- python3 scripts/rebuild_alone.py --updates 20
find $OUT/rb_kstats -name '*kernel_trace.csv' -delete
OPT=lib VALS="default lazystage" REPS=3 CASES="c2_20|--steps 20 --warmup 5;c3_20|--config C3 --steps 20 --warmup 5" bash scripts/ab.sh ${S_OUT:-r06s10}/ab_stage
exit 0
