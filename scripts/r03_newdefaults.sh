#!/bin/bash
# The new N = 1 defaults (4 lanes off the null stream, 12 queues, auto grids 100/lanes + 12 %) on every config, the
# per-frame rebuilds with and without them, the world-1 comm path with 3 / 4 lanes, and the shares at 24 % grids.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/newdef; mkdir -p $OUT
run() { tag=$1; shift; timeout -k 10 300 "$@" --no-cpu-baseline > $OUT/$tag.log 2>&1 || { echo "fail $tag"; tail -3 $OUT/$tag.log; exit 1; }
        echo "$tag: $(grep -o '"ms_per_step": [0-9.]*\|"overlap_lanes": [0-9]*\|"hw_queues": [0-9]*' $OUT/$tag.log | tr '\n' ' ')"; }
for rep in 1 2; do
run c2_$rep python3 bench.py --config C2 --steps 100
run c3_$rep python3 bench.py --config C3 --steps 40
run c4_$rep python3 bench.py --config C4 --steps 100
run c2lbvh_$rep python3 bench.py --config C2 --build lbvh --steps 100
run c5_$rep python3 bench.py --config C5 --build lbvh --steps 12
run c2lbvhrb_$rep python3 bench.py --config C2 --build lbvh --rebuild --steps 100
run c2lbvhrb_new_$rep env RTAMD_HWQ=12 python3 bench.py --config C2 --build lbvh --rebuild --steps 100 --overlap 4 --lane-priority 0
run c5rb_$rep python3 bench.py --config C5 --build lbvh --rebuild --steps 12
run c5rb_new_$rep env RTAMD_HWQ=12 python3 bench.py --config C5 --build lbvh --rebuild --steps 12 --overlap 4 --lane-priority 0
run comm3_$rep python3 bench.py --config C2 --attach-comm --steps 100 --overlap 3
run comm4_$rep python3 bench.py --config C2 --attach-comm --steps 100
run sh08_$rep python3 bench.py --config C2 --shard 0/8 --steps 200
run sh48_$rep python3 bench.py --config C2 --shard 4/8 --steps 200
run c4sh28_$rep python3 bench.py --config C4 --shard 2/8 --steps 200
run sh14_$rep python3 bench.py --config C2 --shard 1/4 --steps 200
done
