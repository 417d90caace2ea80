#!/bin/bash
# Whole-frame lanes off the null stream: lanes x grid_pct (12 queues), and the per-frame rebuild with more reserved
# workgroup slots (option "reserve") beside new-stream lanes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/lanes_new; mkdir -p $OUT
run() { tag=$1; shift; RTAMD_HWQ=12 timeout -k 10 300 python3 bench.py "$@" --no-cpu-baseline > $OUT/$tag.log 2>&1 || { echo "fail $tag"; tail -3 $OUT/$tag.log; exit 1; }
        echo "$tag: $(grep -o '"ms_per_step": [0-9.]*' $OUT/$tag.log)"; }
for rep in 1 2; do
run c2_l3_def_$rep --config C2 --steps 100
run c2_l3_p0_g40_$rep --config C2 --steps 100 --lane-priority 0 --opt grid_pct=40
run c2_l3_p0_g60_$rep --config C2 --steps 100 --lane-priority 0 --opt grid_pct=60
run c2_l4_p0_$rep --config C2 --steps 100 --lane-priority 0 --overlap 4
run c2_l4_p0_g40_$rep --config C2 --steps 100 --lane-priority 0 --overlap 4 --opt grid_pct=40
run c2_l5_p0_g35_$rep --config C2 --steps 100 --lane-priority 0 --overlap 5 --opt grid_pct=35
run c2lbvhrb_p0_res64_$rep --config C2 --build lbvh --rebuild --steps 100 --lane-priority 0 --opt reserve=64
run c2lbvhrb_p0_res128_$rep --config C2 --build lbvh --rebuild --steps 100 --lane-priority 0 --opt reserve=128
run c5rb_p0_res64_$rep --config C5 --build lbvh --rebuild --steps 12 --lane-priority 0 --opt reserve=64
done
