#!/bin/bash
# Round-2 sweeps on one GPU: overlap lanes x reserve, threshold, and the C4 per-rank shares.
# usage: sweep_r02.sh [what]  (what: lanes | thr | c4 | reorder | split | period | period2 | shares | all; outputs gpurun_out/sweep_*.jsonl)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
WHAT=${1:-all}
one() {  # out args...
  local out=$1; shift
  timeout -k 10 240 python bench.py --no-cpu-baseline "$@" > gpurun_out/_one.log 2>&1
  local rc=$?
  if [ $rc -ne 0 ]; then echo "rc=$rc for $*"; tail -3 gpurun_out/_one.log; exit $rc; fi
  tail -1 gpurun_out/_one.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'args': '$*', 'hwq': '${GPU_MAX_HW_QUEUES:-}', 'value': d['value'], 'ms_per_step': d['ms_per_step'], 'kernel_ms': d['kernel_ms'], 'kernel_ms_overlapped': d['kernel_ms_overlapped'], 'lat': d['frame_latency_ms_median'], 'host_update_ms': d.get('host_update_ms_median'), 'host_wait_ms': d.get('host_update_wait_ms_median'), 'host_call_ms': d.get('host_call_ms_median'), 'host_busy_ms': d.get('host_busy_ms_median')}))" | tee -a "gpurun_out/$out"
}
if [[ $WHAT == lanes || $WHAT == all ]]; then
  for rep in 1 2; do for L in 2 3 4; do for rs in 0 8 16; do one sweep_lanes.jsonl --overlap $L --opt reserve=$rs; done; done; done
fi
if [[ $WHAT == queues ]]; then
  # hardware queues per process (GPU_MAX_HW_QUEUES, HIP default 4) x overlap lanes: full C2 frame and 1/8 shares
  for rep in 1; do for hq in 4 8; do for L in 3 4 6 8; do
    GPU_MAX_HW_QUEUES=$hq one sweep_queues.jsonl --overlap $L --steps 200
    GPU_MAX_HW_QUEUES=$hq one sweep_queues.jsonl --overlap $L --steps 200 --shard 4/8
    GPU_MAX_HW_QUEUES=$hq one sweep_queues.jsonl --overlap $L --steps 200 --config C4 --shard 3/8
  done; done; done
fi
if [[ $WHAT == grid ]]; then
  # option "grid_pct": each overlapped launch takes only part of the GPU, so more than two lanes' launches
  # run side by side (hardware queues raised to 8 so every lane has its own)
  for lp in 3:100 3:50 4:50 6:35 6:50 8:25 8:35; do L=${lp%:*}; P=${lp#*:}
    GPU_MAX_HW_QUEUES=8 one sweep_grid.jsonl --overlap $L --opt grid_pct=$P --steps 200 --shard 4/8
    GPU_MAX_HW_QUEUES=8 one sweep_grid.jsonl --overlap $L --opt grid_pct=$P --steps 200 --config C4 --shard 3/8
    GPU_MAX_HW_QUEUES=8 one sweep_grid.jsonl --overlap $L --opt grid_pct=$P --steps 200
  done
fi
if [[ $WHAT == grid2 ]]; then
  # finer grid_pct x lanes at the default 4 hardware queues; the full C2 frame is the bench line
  for rep in 1 2; do for lp in 3:100 3:50 3:60 3:67 4:34 4:50 4:60 5:40; do L=${lp%:*}; P=${lp#*:}
    one sweep_grid2.jsonl --overlap $L --opt grid_pct=$P --steps 200
    one sweep_grid2.jsonl --overlap $L --opt grid_pct=$P --steps 200 --shard 4/8
    one sweep_grid2.jsonl --overlap $L --opt grid_pct=$P --steps 200 --config C4 --shard 3/8
  done; done
  for lp in 3:100 3:50 4:50; do L=${lp%:*}; P=${lp#*:}; one sweep_grid2.jsonl --overlap $L --opt grid_pct=$P --config C3; done
fi
if [[ $WHAT == shares2 ]]; then
  # every 1/8 share of C2 and C4 with the library defaults (3 lanes, auto grid_pct), and the full frames
  one sweep_shares2.jsonl --steps 200
  one sweep_shares2.jsonl --steps 200 --config C4
  for r in 0 1 2 3 4 5 6 7; do
    one sweep_shares2.jsonl --steps 200 --shard $r/8
    one sweep_shares2.jsonl --steps 200 --config C4 --shard $r/8
  done
  for L in 2 3; do one sweep_shares2.jsonl --steps 200 --overlap $L --opt grid_pct=50; one sweep_shares2.jsonl --steps 200 --overlap $L --opt grid_pct=50 --shard 1/8; done
fi
if [[ $WHAT == claim ]]; then
  # option "claim_items": order items per queue atomic (1 vs 2), alternating
  for rep in 1 2; do for v in 1 2; do
    one sweep_claim.jsonl --opt claim_items=$v
    one sweep_claim.jsonl --opt claim_items=$v --shard 4/8
    one sweep_claim.jsonl --opt claim_items=$v --config C3
    one sweep_claim.jsonl --opt claim_items=$v --config C4 --shard 3/8
  done; done
fi
if [[ $WHAT == mix ]]; then
  # option "mix": per refill the heaviest item from the band's front, light fill from its back
  for rep in 1 2; do for v in 0 1; do
    one sweep_mix.jsonl --opt mix=$v
    one sweep_mix.jsonl --opt mix=$v --shard 4/8
    one sweep_mix.jsonl --opt mix=$v --config C3
    one sweep_mix.jsonl --opt mix=$v --config C4 --shard 3/8
  done; done
fi
if [[ $WHAT == lds2 ]]; then
  # option "lds_scene" 1 (TLAS quads + instance hot records) vs 2 (also analytic primitives + instance cold records)
  for rep in 1 2; do for v in 1 2; do
    one sweep_lds2.jsonl --opt lds_scene=$v
    one sweep_lds2.jsonl --opt lds_scene=$v --shard 4/8
    one sweep_lds2.jsonl --opt lds_scene=$v --config C3
    one sweep_lds2.jsonl --opt lds_scene=$v --build lbvh
  done; done
fi
if [[ $WHAT == drain ]]; then
  # option "drain": after a wave's queue is dry, shade when 1/drain of its remaining paths wait
  for rep in 1 2; do for v in ${DRAIN_VALUES:-0 1 2 4 64}; do
    one sweep_drain.jsonl --opt drain=$v --overlap 1
    one sweep_drain.jsonl --opt drain=$v
    one sweep_drain.jsonl --opt drain=$v --shard 4/8
    one sweep_drain.jsonl --opt drain=$v --config C3
  done; done
fi
if [[ $WHAT == group ]]; then
  # option "group": instances with identical transforms share one SAH BLAS (one TLAS item)
  for rep in 1 2; do for v in 0 1; do
    one sweep_group.jsonl --pre-opt group=$v --overlap 1
    one sweep_group.jsonl --pre-opt group=$v
    one sweep_group.jsonl --pre-opt group=$v --shard 4/8
    one sweep_group.jsonl --pre-opt group=$v --config C3
    one sweep_group.jsonl --pre-opt group=$v --config C4 --shard 3/8
  done; done
fi
if [[ $WHAT == host ]]; then
  # host-side time per pipelined frame (host_busy: the rt_render call minus its waits on the GPU)
  one sweep_host.jsonl
  one sweep_host.jsonl --shard 4/8
  one sweep_host.jsonl --config C4 --shard 3/8
  one sweep_host.jsonl --overlap 1 --shard 4/8
fi
if [[ $WHAT == lanes8 ]]; then
  # many frames in flight for a rank's share: L lanes x P % grids, 8 hardware queues
  for lp in 3:0 6:15 8:12 8:15 8:20; do L=${lp%:*}; P=${lp#*:}
    GPU_MAX_HW_QUEUES=8 one sweep_lanes8.jsonl --overlap $L --opt grid_pct=$P --steps 200 --shard 4/8
  done
  for lp in 8:12 8:25; do L=${lp%:*}; P=${lp#*:}
    GPU_MAX_HW_QUEUES=8 one sweep_lanes8.jsonl --overlap $L --opt grid_pct=$P --steps 200
  done
fi
if [[ $WHAT == ldsblas ]]; then
  # option "lds_blas": the group BLAS's top levels in the LDS scene region
  for rep in 1 2; do for v in 0 1; do
    one sweep_ldsblas.jsonl --opt lds_blas=$v
    one sweep_ldsblas.jsonl --opt lds_blas=$v --overlap 1
    one sweep_ldsblas.jsonl --opt lds_blas=$v --shard 4/8
    one sweep_ldsblas.jsonl --opt lds_blas=$v --config C3
  done; done
fi
if [[ $WHAT == lanes8b ]]; then
  # frames in flight for a rank's share after one completion event per launch: lanes x grid share x hw queues
  for cfg in "4:0:4" "4:0:8" "6:0:8" "6:20:8" "8:15:8" "8:0:8"; do IFS=: read L P Q <<< "$cfg"
    GPU_MAX_HW_QUEUES=$Q one sweep_lanes8b.jsonl --overlap $L --opt grid_pct=$P --steps 200 --shard 4/8
  done
  for cfg in "4:0:4" "4:0:8" "6:0:8"; do IFS=: read L P Q <<< "$cfg"
    GPU_MAX_HW_QUEUES=$Q one sweep_lanes8b.jsonl --overlap $L --opt grid_pct=$P --steps 200
    GPU_MAX_HW_QUEUES=$Q one sweep_lanes8b.jsonl --overlap $L --opt grid_pct=$P --steps 200 --config C4 --shard 3/8
  done
  one sweep_lanes8b.jsonl --steps 200 --config C4 --shard 3/8
  one sweep_lanes8b.jsonl --steps 200 --config C4
fi
if [[ $WHAT == shares3 ]]; then
  # share defaults of bench.py (6 lanes, 20 % grids, 8 hardware queues) over several ranks, and the full frames
  for r in 0 2 4 6; do one sweep_shares3.jsonl --steps 200 --shard $r/8; one sweep_shares3.jsonl --steps 200 --config C4 --shard $r/8; done
  one sweep_shares3.jsonl --steps 200 --config C4
  one sweep_shares3.jsonl --steps 200
fi
if [[ $WHAT == retune ]]; then
  # knobs re-checked after lds_scene / grid_pct / chained root leaves: refill threshold, split levels, reorder period
  for rep in 1 2; do
    for t in 24 32 40 48 56; do one sweep_retune.jsonl --threshold $t; done
    for sp in 2572 3084 3598 65535; do one sweep_retune.jsonl --opt split=$sp; done
    for k in 4 16; do one sweep_retune.jsonl --opt reorder_period=$k; done
    for t in 24 40; do one sweep_retune.jsonl --threshold $t --shard 4/8; done
    one sweep_retune.jsonl --shard 4/8
  done
fi
if [[ $WHAT == retune2 ]]; then
  # knobs re-checked after groups / flat quads / reciprocal slabs / one event per launch, pipelined and serialised
  for rep in 1 2; do for ov in "" "--overlap 1"; do
    for t in 24 32 40 48; do one sweep_retune2.jsonl --threshold $t $ov; done
    for sp in 2572 3598 65535; do one sweep_retune2.jsonl --opt split=$sp $ov; done
    for k in 4 16; do one sweep_retune2.jsonl --opt reorder_period=$k $ov; done
  done; done
fi
if [[ $WHAT == thr2 ]]; then
  # refill threshold 32..64 after the session-3 changes: full frame, serialised, a share, C3
  for rep in 1 2; do for t in 32 40 48 56 64; do
    one sweep_thr2.jsonl --threshold $t
    one sweep_thr2.jsonl --threshold $t --overlap 1
    one sweep_thr2.jsonl --threshold $t --shard 4/8
    one sweep_thr2.jsonl --threshold $t --config C3
  done; done
fi
if [[ $WHAT == thrauto ]]; then
  # auto threshold (64 at depth x spp <= 2, else 40) vs 32 on the other configurations
  for rep in 1 2; do for t in 32 0; do
    one sweep_thrauto.jsonl --threshold $t --config C4
    one sweep_thrauto.jsonl --threshold $t --config C4 --shard 3/8
    one sweep_thrauto.jsonl --threshold $t --shard 0/8
    one sweep_thrauto.jsonl --threshold $t --build lbvh
  done; done
  for t in 32 0; do one sweep_thrauto.jsonl --threshold $t --config C5 --build lbvh --rebuild --steps 20 --warmup 3; done
fi
if [[ $WHAT == order2 ]]; then
  # claim-order knobs under the auto threshold: merged light pairs, heavy-unit quarters
  for rep in 1 2; do for o in "--opt merge=0" "--opt merge=6" "--opt merge=8" "--opt split=65535" "--opt split=2570"; do
    one sweep_order2.jsonl $o
    one sweep_order2.jsonl $o --overlap 1
    one sweep_order2.jsonl $o --shard 4/8
  done; done
fi
if [[ $WHAT == drain2 ]]; then
  # option "drain" under the auto threshold (64 for C2: a wave otherwise shades only when all its lanes are idle)
  for rep in 1 2; do for v in 0 2 4 16; do
    one sweep_drain2.jsonl --opt drain=$v
    one sweep_drain2.jsonl --opt drain=$v --overlap 1
    one sweep_drain2.jsonl --opt drain=$v --shard 4/8
  done; done
fi
if [[ $WHAT == leaf2 ]]; then
  # SAH BLAS leaf size with instance groups and the auto threshold
  for rep in 1 2; do for v in 2 3 4; do
    one sweep_leaf2.jsonl --pre-opt blas_leaf=$v
    one sweep_leaf2.jsonl --pre-opt blas_leaf=$v --overlap 1
    one sweep_leaf2.jsonl --pre-opt blas_leaf=$v --shard 4/8
    one sweep_leaf2.jsonl --pre-opt blas_leaf=$v --config C3
  done; done
fi
if [[ $WHAT == tile2 ]]; then
  # screen-tile edge for the rank shares (balance of the slowest share)
  for t in 32 64; do for r in 0 2 4 6; do
    one sweep_tile2.jsonl --steps 200 --shard $r/8 --tile $t
    one sweep_tile2.jsonl --steps 200 --config C4 --shard $r/8 --tile $t
  done; done
fi
if [[ $WHAT == lanes3 ]]; then
  # whole-frame lanes x reserve after the session-3 changes
  for rep in 1 2; do for cfg in "3 16" "3 0" "3 8" "2 16" "4 16"; do set -- $cfg
    one sweep_lanes3.jsonl --overlap $1 --opt reserve=$2
  done; done
fi
if [[ $WHAT == lanes8c ]]; then
  # more frames in flight for a share (after one event per launch, auto threshold, 32x32 tiles)
  for cfg in "6:20:8" "8:15:8" "8:15:12" "8:12:12" "7:17:12"; do IFS=: read L P Q <<< "$cfg"
    GPU_MAX_HW_QUEUES=$Q one sweep_lanes8c.jsonl --overlap $L --opt grid_pct=$P --steps 200 --shard 4/8 --tile 32
    GPU_MAX_HW_QUEUES=$Q one sweep_lanes8c.jsonl --overlap $L --opt grid_pct=$P --steps 200 --config C4 --shard 2/8 --tile 32
  done
fi
if [[ $WHAT == lanes4 ]]; then
  # whole frame: lanes with the lane-scaled auto grid and more hardware queues
  for rep in 1 2; do for cfg in "3:4" "4:12" "5:12" "6:12" "8:12"; do IFS=: read L Q <<< "$cfg"
    GPU_MAX_HW_QUEUES=$Q one sweep_lanes4.jsonl --overlap $L
  done; done
fi
if [[ $WHAT == order3 ]]; then
  # claim-order cost and period under the auto threshold
  for rep in 1 2; do for o in "--opt cost_max=0" "--opt cost_max=1" "--opt reorder_period=4" "--opt reorder_period=16"; do
    one sweep_order3.jsonl $o
    one sweep_order3.jsonl $o --overlap 1
    one sweep_order3.jsonl $o --shard 4/8
  done; done
fi
if [[ $WHAT == costmax ]]; then
  # option "cost_max": claim order by a unit's longest path (x 64) instead of its summed cost; split levels
  for rep in 1 2; do for o in "--opt cost_max=0" "--opt cost_max=1" "--opt cost_max=1 --opt split=3598" "--opt cost_max=1 --opt split=65535"; do
    one sweep_costmax.jsonl $o
    one sweep_costmax.jsonl $o --shard 4/8
    one sweep_costmax.jsonl $o --config C3
  done; done
fi
if [[ $WHAT == merge ]]; then
  # option "merge": adjacent light units share one claim item (levels below the value)
  for rep in 1 2; do for v in 0 6 8 10; do
    one sweep_merge.jsonl --opt merge=$v
    one sweep_merge.jsonl --opt merge=$v --shard 4/8
    one sweep_merge.jsonl --opt merge=$v --config C3
  done; done
fi
if [[ $WHAT == lds ]]; then
  # option "lds_scene": TLAS quads + instance hot records in LDS (1) vs HBM (0), alternating
  for rep in 1 2; do for v in 0 1; do
    one sweep_lds.jsonl --opt lds_scene=$v
    one sweep_lds.jsonl --opt lds_scene=$v --shard 4/8
    one sweep_lds.jsonl --opt lds_scene=$v --config C4 --shard 3/8
    one sweep_lds.jsonl --opt lds_scene=$v --config C3
    one sweep_lds.jsonl --opt lds_scene=$v --build lbvh
  done; done
fi
if [[ $WHAT == thr || $WHAT == all ]]; then
  for t in 24 32 40 48; do one sweep_thr.jsonl --threshold $t ${THR_ARGS:-}; done
fi
if [[ $WHAT == c4 || $WHAT == all ]]; then
  one sweep_c4.jsonl --config C4 ${C4_ARGS:-}
  for r in 0 1 2 3 4 5 6 7; do one sweep_c4.jsonl --config C4 --shard $r/8 ${C4_ARGS:-}; done
fi
if [[ $WHAT == split ]]; then
  # heavy-first order with / without split claims vs screen order
  for rep in 1 2; do for o in "--opt reorder=0" "--opt reorder=1" "--opt reorder=1 --opt split=0xFFFF" "--opt reorder=1 --opt split=0x0C0C"; do
    one sweep_split.jsonl $o
    one sweep_split.jsonl --config C3 $o
  done; done
fi
if [[ $WHAT == period ]]; then
  # reorder period K (costs recorded / order rebuilt once per K launches of a lane) x split claims
  for rep in 1 2; do for o in "--opt reorder=0" "--opt reorder_period=1" "--opt reorder_period=8" "--opt reorder_period=8 --opt split=0xFFFF" "--opt reorder_period=32 --opt split=0xFFFF"; do
    one sweep_period.jsonl $o
  done; done
  for o in "--opt reorder=0" "--opt reorder_period=1" "--opt reorder_period=8" "--opt reorder_period=8 --opt split=0xFFFF"; do
    one sweep_period.jsonl --config C3 $o
    one sweep_period.jsonl --config C4 --shard 3/8 $o
  done
fi
if [[ $WHAT == lanes4 ]]; then
  for L in 3 4; do
    one sweep_lanes4.jsonl --overlap $L
    one sweep_lanes4.jsonl --config C2 --shard 4/8 --overlap $L
    one sweep_lanes4.jsonl --config C4 --shard 4/8 --overlap $L
    one sweep_lanes4.jsonl --config C4 --overlap $L
  done
fi
if [[ $WHAT == shares ]]; then
  # N=1 frame and each rank's 1/8 share (64x64 tiles) of C4 and C2 with the library defaults
  for cfg in C4 C2; do
    one sweep_shares.jsonl --config $cfg
    for r in 0 1 2 3 4 5 6 7; do one sweep_shares.jsonl --config $cfg --shard $r/8; done
  done
fi
if [[ $WHAT == period2 ]]; then
  for rep in 1 2; do for o in "--opt reorder_period=1 --opt split=0x0C0C" "--opt reorder_period=4 --opt split=0x0C0C" "--opt reorder_period=8 --opt split=0x0C0C"; do
    one sweep_period2.jsonl $o
  done; done
  for o in "--opt reorder_period=4 --opt split=0x0C0C" "--opt reorder_period=8 --opt split=0x0C0C"; do
    one sweep_period2.jsonl --config C3 $o
    one sweep_period2.jsonl --config C4 --shard 3/8 $o
  done
fi
if [[ $WHAT == reorder ]]; then
  # claim order on/off across the configs (heaviest-first order vs screen order)
  for rep in 1 2; do for ro in 0 1; do
    one sweep_reorder.jsonl --opt reorder=$ro
    one sweep_reorder.jsonl --config C3 --opt reorder=$ro
  done; done
  for ro in 0 1; do for r in 0 3 5 7; do one sweep_reorder.jsonl --config C4 --shard $r/8 --opt reorder=$ro; done; done
  for ro in 0 1; do one sweep_reorder.jsonl --config C5 --build lbvh --rebuild --steps 8 --warmup 2 --opt reorder=$ro; done
fi
exit 0
