#!/usr/bin/env python3
"""Benchmark: Mrays/s + ms/frame of the trace path on BASELINE.json config C2.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    (N > 1: python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 ... bench.py --gpus N)

A step is one frame of the reference's render loop (src/Global/Renderer.cu:264-317): the
instance update callback (Main.cu updateInstance, native), the host TLAS rebuild + upload,
and the trace kernel over the frame — for N > 1 each rank traces its interleaved 32x32
screen tiles, and the library gathers the tiles to rank 0 over RCCL and assembles the frame there,
inside rt_render (rt_scene_attach_comm; torch.distributed only broadcasts the RCCL id and runs the
barriers and the max-over-ranks timing).  Scene, BVHs and framebuffer stay in HBM; nothing is
copied to the host inside the timed region.

Rank 0 prints one JSON line (see DESIGN.md §4 for every field's definition).
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "real-time-gpu-ray-tracer_amd"))

METRIC = "Mrays/sec + ms/frame, 1920×1080 1spp primary+shadow, 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
TILE = 32

# SURVEY §8(d) algorithmic bytes (the roofline's `achieved`):
#   B = 32 N_aabb + 36 N_tri + 32 N_sph_or_quad + 48 N_inst + 32 per ray (state in/out) + 4 per pixel
A_AABB, A_TRI, A_SQ, A_INST, A_RAY, A_PIXEL = 32, 36, 32, 48, 32, 4
# bytes the kernel's own layout moves per item (reported beside, never as `achieved`)
B_PAIR, B_TRI, B_SPH, B_QUAD, B_INST, B_HIT, B_PIXEL = 64, 48, 16, 80, 80, 208, 4
# measured HBM fraction below which the kernel is reported latency-bound
LATENCY_BOUND_FRAC = 0.25
PMC_DIR = os.path.join(REPO, "profiles", "pmc")


# width, height, requested spp per config (read before HIP starts; checked against rtamd.scenes.CONFIGS in main)
FRAME_DIMS = {"C1": (256, 256, 1), "C2": (1920, 1080, 1), "C3": (1920, 1080, 4), "C4": (1920, 1080, 1),
              "C5": (3840, 2160, 8)}


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=100)
    p.add_argument("--warmup", type=int, default=10)
    p.add_argument("--config", default="C2")
    p.add_argument("--exact", action="store_true", help="time the EXACT (parity) kernel instead of FAST")
    p.add_argument("--build", default="sah", choices=("sah", "compat", "lbvh"),
                   help="BVH builder: SAH (default), the reference's random-axis median split, or the GPU LBVH builder")
    p.add_argument("--rebuild", action="store_true", help="--build lbvh: rebuild every BLAS on the GPU each frame (C5)")
    p.add_argument("--no-rebuild-roofline", action="store_true",
                   help="--rebuild: skip the untimed rebuild-alone stage timing (the line's \"rebuild\" block)")
    p.add_argument("--kernel", type=int, default=1, help="1 = persistent megakernel, 0 = grid kernel")
    p.add_argument("--overlap", type=int, default=None,
                   help="L >= 2: consecutive frames cycle L streams / library lanes so frame k+1 fills the CUs "
                        "frame k's tail leaves idle; 0 or 1: frames are serialised (default 3)")
    p.add_argument("--lanes", default="library", choices=("library", "caller"),
                   help="library: frames without a stream on lanes the scene owns (option overlap -1 picks the lane "
                        "count and staging depth; --overlap L sets L); caller: bench creates the lane streams")
    p.add_argument("--lane-priority", type=int, default=None,
                   help="overlap lanes on new HIP streams of this priority (torch: -1 high, 0 normal); default: "
                        "new normal-priority streams, except the current stream + new ones with a per-frame rebuild")
    p.add_argument("--shard", default=None, help="R/N: trace only rank R's tiles of an N-rank split on this one GPU "
                                                 "(per-rank cost study; no gather)")
    p.add_argument("--opt", action="append", default=[], help="extra rt_scene_set_option key=value (A/B studies)")
    p.add_argument("--pre-opt", action="append", default=[], help="rt_scene_set_option key=value before the build")
    # 32: the ranks' shares balance better than with 64 (slowest C4 1/8 share 0.064 -> 0.059 ms/frame, C2
    # equal; profiles/r02_sweep_tile2.jsonl)
    p.add_argument("--tile", type=int, default=32, help="N > 1 screen-tile edge in pixels (multiple of 8)")
    p.add_argument("--attach-comm", action="store_true",
                   help="N = 1: run the multi-GPU frame path anyway (a world-1 RCCL communicator: tiles + assemble)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-seconds", type=float, default=12.0)
    p.add_argument("--clock-warmup", type=float, default=0.5,
                   help="seconds of untimed frames before the W warm-up steps (the GPU's clocks ramp up under load)")
    p.add_argument("--print-pmc-tag", action="store_true", help="print this run's PMC tag as JSON and exit (no GPU)")
    p.add_argument("--skip-update", action="store_true",
                   help="diagnostic: timed frames reuse the last frame block (no host update / upload); images are stale")
    p.add_argument("--launch-times", default=None,
                   help="write the timed launches' (start, stop) ms, relative to the first start, to this .npy (diagnostic)")
    return p.parse_args()


def algorithmic_bytes(st):
    """the bytes a ray's tests must read, independent of this kernel's layout."""
    return (A_AABB * st["aabb_tests"] + A_TRI * st["triangle_tests"] + A_SQ * st["sphere_quad_tests"] +
            A_INST * st["instance_visits"] + A_RAY * st["rays"] + A_PIXEL * st["pixels"])


def layout_bytes(st):
    """Bytes this kernel's records occupy per item (64 B node pair, 48 B TriHot, 80 B InstHot, ...)."""
    spheres = st["sphere_quad_tests"] - st["quad_tests"]
    return (B_PAIR * st["aabb_tests"] / 2 + B_TRI * st["triangle_tests"] + B_SPH * spheres +
            B_QUAD * st["quad_tests"] + B_INST * st["instance_visits"] + B_HIT * st["hits"] +
            B_PIXEL * st["pixels"])


def host_cores():
    """Cores this process may run on: the affinity mask, capped by a cgroup CPU quota if one is set
    (os.cpu_count() on the GPU box reports the whole machine, not this job's share)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            quota, period = f.read().split()[:2]
        if quota != "max":
            n = min(n, max(1, int(int(quota) // int(period))))
    except (OSError, ValueError):
        pass
    return max(1, n)


def cpu_baseline(scene, cfg, budget_s):
    """The oracle ("port": oracle/rt_oracle.c, the reference's algorithm restated in C) on the host:
    whole frames of the same scene, camera and seed, repeated until ~budget_s on every core this job
    may use, then ~budget_s / 2 on one core.  It traces the reference's own trees (random-axis median
    split, RT_BUILD_COMPAT_MEDIAN), which is what the reference's CPU path would trace; the GPU leg
    traces SAH trees of the same primitives (same closest hits up to 1e-6 ties, fewer node visits)."""
    from oracle.oracle import OracleScene
    o = OracleScene(scene, build_seed=0)
    o.camera(cfg.width, cfg.height)

    def run(threads, budget):
        rays = frames = 0
        t0 = time.perf_counter()
        while True:
            o.update(frames)
            _, _, cnt = o.render(threads=threads, want_rgb=False, want_rgba=True)
            rays += cnt["rays"]
            frames += 1
            if time.perf_counter() - t0 >= budget:
                break
        return rays, frames, time.perf_counter() - t0

    threads = host_cores()
    rays, frames, dt = run(threads, budget_s)
    rays1, frames1, dt1 = run(1, budget_s / 2)
    return {"value": round(rays / dt / 1e6, 3), "unit": "Mrays/s", "cores": threads, "kind": "port",
            "sample": f"oracle/rt_oracle.c, {frames} full {cfg.width}x{cfg.height} {cfg.name} frames "
                      f"(frames 0..{frames - 1}), {threads} threads, {dt:.1f} s, {rays} rays; "
                      f"reference median-split trees (compat build, seed 0)",
            "ms_per_frame": round(dt * 1e3 / frames, 2),
            "one_core": {"value": round(rays1 / dt1 / 1e6, 3), "unit": "Mrays/s", "cores": 1,
                         "ms_per_frame": round(dt1 * 1e3 / frames1, 2),
                         "sample": f"{frames1} frames, {dt1:.1f} s, {rays1} rays"},
            "trees": "compat (reference random-axis median split)"}


def lib_sha16():
    """Identity of the trace library this run loads (the PMC summaries are tagged with it)."""
    from rtamd import abi
    path = os.environ.get("RTAMD_LIB") or abi.LIB_PATH
    with open(path, "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()[:16]


def build_provenance():
    """The library's build stamp (rtamd/provenance.py): sources hash and the git HEAD that built it."""
    from rtamd import provenance
    ok, msg = provenance.check()
    try:
        with open(provenance.STAMP) as f:
            d = json.load(f)
    except (OSError, ValueError):
        d = {}
    return {"stamp_ok": ok, "sources_sha16": (d.get("sources_sha256") or "")[:16], "git_head": d.get("git_head"),
            "dirty_at_build": d.get("sources_dirty_at_build")}


def pmc_tag(args):
    """What a PMC summary must have been measured on to price this run's launches: the same config, BVH
    builder, per-frame rebuild, kernel (EXACT / FAST, persistent / grid), scene options and library build."""
    return {"config": args.config, "build": args.build, "rebuild": bool(args.rebuild), "exact": bool(args.exact),
            "kernel": int(args.kernel), "options": sorted(args.pre_opt + args.opt), "lib_sha16": lib_sha16()}


def pmc_path(tag):
    return os.path.join(PMC_DIR, f"{tag['config']}_{tag['build']}{'_rebuild' if tag['rebuild'] else ''}"
                                 f"{'_exact' if tag['exact'] else ''}{'' if tag['kernel'] else '_grid'}.json")


def load_traffic(tag):
    """HBM bytes per launch (2 x FETCH_SIZE + WRITE_SIZE, MI355X_MICROARCH.md's gfx950 correction) of the trace
    kernel from the committed rocprofv3 PMC summary of this exact workload (scripts/pmc_tagged.sh writes
    profiles/pmc/<config>_<build>....json): only if every tag field, the library hash included, matches.
    Returns (bytes or None, summary path or None, why)."""
    path = pmc_path(tag)
    try:
        with open(path) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None, None, f"no PMC summary {os.path.relpath(path, REPO)}"
    diff = [k for k, v in tag.items() if d.get("tag", {}).get(k) != v]
    if diff:
        return None, None, f"{os.path.relpath(path, REPO)} measured another workload or build ({', '.join(diff)} differ)"
    return d.get("hbm_bytes_per_launch"), os.path.relpath(path, REPO), "tagged PMC summary"


rt_scene_lanes_max = 8                                     # rt.h: "overlap" lanes 2..8


# The per-frame GPU BLAS rebuild (--build lbvh --rebuild; csrc/lbvh.hip) priced per stage the way the trace is: the
# bytes each stage's kernels must move at least (reads of their inputs, writes of their outputs, per item / interior
# node / node pair of the forest; scratch and re-reads not counted), over the stage's HIP-event time in a rebuild alone
# (option "timeline": events between the stages, rt_scene_debug_read "rebuild_stages").  N items (10 M triangles on
# C5), NI = N - trees interior nodes, P node pairs written (interior nodes of > 4 items).
REBUILD_STAGES = ("prep", "bounds", "morton", "sort", "hierarchy_small", "hierarchy_large", "scan", "emit_roots",
                  "collapse")


def rebuild_bytes(N, NI, P, NL, TL):
    """Algorithmic bytes per builder stage (csrc/lbvh.hip) of a rebuild over N items, NI interior nodes, P node pairs,
    NL of the items in TL large trees (> 2048 items: rocPRIM sort, hierarchy_chunk_kernel / hierarchy_top_kernel)."""
    NS, NIL = N - NL, max(NL - TL, 0)
    NIS = max(NI - NIL, 0)
    return {
        # 36 B vertices + segment id + group member read; 24 B box, 16 B centroid, 48 B TriHot staged (item order)
        "prep": N * (36 + 4 + 4 + 24 + 16 + 48),
        "bounds": N * (16 + 4),                                # centroid + segment id
        "morton": N * (16 + 4 + 4 + 4),                        # centroid + segment id in, key + item out
        # small trees: one LDS pass (key + item in and out); large: key histogram + three 10-bit passes
        "sort": NS * 16 + NL * (4 + 3 * 16),
        # small trees: Karras (sorted key, segment id, item id; child / range / flag / parent per node), the leaf-
        # ordered gather (staged 48 B record in, 48 B out), the LDS bottom-up (item box by id, parent per item; per node
        # children, range, parent in, box, height, kept flag out)
        "hierarchy_small": NS * (4 + 4 + 4 + 48 + 48 + 24 + 4 + 4) + NIS * (8 + 8 + 4 + 8 + 8 + 8 + 4 + 24 + 4 + 4),
        # large trees, one bottom-up climb: sorted key, segment id, item id, item box (24) per item; children, range,
        # box, height, kept flag out per node; the gather (staged 48 B record in, 48 B out)
        "hierarchy_large": NL * (4 + 4 + 4 + 24 + 48 + 48) + NIL * (8 + 8 + 24 + 4 + 4),
        "scan": NI * 8,                                        # kept flags in, pair indices out
        # kept flag per node; per pair: children, range, segment, two child boxes, child pair indices, 64 B pair out
        "emit_roots": NI * 4 + P * (8 + 8 + 4 + 48 + 8 + 64),
        "collapse": P * (64 + 128 + 128),                      # own pair + <= 2 child pairs in, 128 B quad out
    }


def rebuild_roofline(r, frames):
    """Rebuild-alone timing of the scene's per-frame BLAS rebuild (rt_scene_update, no trace) with stage events: mean
    stage ms over `frames` updates, algorithmic bytes per stage, achieved GB/s and the fraction of HBM peak; the chain
    total too.  Called after the timed region (events between the stages cost ~5 us each)."""
    import numpy as np
    r.set_option("timeline", 1)
    rows = []
    t0 = time.perf_counter()
    for f in frames:
        r.update(f)
        rows.append(r.debug_read("rebuild_stages").view(np.float64).copy())
    wall = (time.perf_counter() - t0) * 1e3 / len(frames)
    r.set_option("timeline", 0)
    a = np.mean(np.stack(rows), axis=0)
    N, NI, P, NL, TL = int(a[0]), int(a[1]), int(round(a[2])), int(a[3]), int(a[4])
    ms = dict(zip(REBUILD_STAGES, a[5:].tolist()))
    by = rebuild_bytes(N, NI, P, NL, TL)
    stages = {k: {"ms": round(ms[k], 4), "bytes": int(by[k]), "achieved_gbs": round(by[k] / (ms[k] * 1e-3) / 1e9, 1),
                  "frac": round(by[k] / (ms[k] * 1e-3) / 1e9 / HBM_PEAK_GBS, 3)} for k in REBUILD_STAGES}
    tot_ms, tot_b = float(sum(ms.values())), float(sum(by.values()))
    return {"items": N, "interior_nodes": NI, "node_pairs": P, "large_tree_items": NL, "updates": len(frames),
            "ms_stages_sum": round(tot_ms, 4), "ms_per_update_wall": round(wall, 4), "bytes": int(tot_b),
            "achieved_gbs": round(tot_b / (tot_ms * 1e-3) / 1e9, 1),
            "frac": round(tot_b / (tot_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 3), "peak_gbs": HBM_PEAK_GBS,
            "timing": "rebuild alone (rt_scene_update, no trace), HIP events between the builder's stages, mean over "
                      "the updates", "stages": stages}


def main():
    args = parse()
    if args.print_pmc_tag:
        print(json.dumps(pmc_tag(args)))
        return
    if not 1 <= args.steps <= 256:
        raise SystemExit("--steps must be in 1..256 (the library's per-frame kernel-time ring)")
    global TILE
    TILE = args.tile
    if TILE % 8 or TILE <= 0:
        raise SystemExit("--tile must be a positive multiple of 8")
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus != world and world > 1:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE {world}")
    n = max(1, world)
    # a rank's 1/N share (N > 1, or the one-GPU --shard study) is bounded by its longest paths, not by its
    # work: more frames in flight pay there (8 lanes with 15 % grids (25 % since round 3) and 12 hardware queues per process, so
    # every lane and the RCCL communicators' streams get queues of their own: C2 1/8 share 0.067 -> 0.045
    # ms/frame, C4 0.090 -> 0.054; profiles/r02_sweep_lanes8b.jsonl, r02_sweep_lanes8c.jsonl).  A whole frame on
    # one GPU: 4 lanes off the null stream with 12 queues (C2 0.173 -> 0.164 ms/frame, C3 1.44 -> 1.39, C4 0.197 ->
    # 0.190; profiles/r03_session2/lanes_new*.txt), except with a per-frame rebuild (below).  Set before HIP starts.
    share = n > 1 or args.shard is not None
    # a per-frame BLAS rebuild overlaps the traces differently: C2-LBVH's runs 0.50 -> 1.0 ms/frame on lanes off the
    # null stream (the rebuild kernels wait behind the lanes' grids), so those frames keep 3 lanes, the null stream
    # as lane 0 and 4 queues (profiles/r03_session2/lane_streams_*.txt, scene_stream_priority_*.txt)
    # ... but not a launch of >= 16 M camera paths (C5): the rebuild kernels then sat behind lane 0's traces in the null
    # stream's hardware queue, and lanes off it run C5 with the rebuild 10.5-10.8 -> 9.7-9.8 ms/frame
    # (profiles/r04/c5_rebuild/r04s16_*)
    w, h, spp = FRAME_DIMS[args.config]
    big = w * h * int(spp ** 0.5) ** 2 >= (16 << 20)
    classic = args.lanes == "caller" and not share and not args.attach_comm and args.rebuild and not big
    # with a communicator attached (N > 1, --attach-comm) RCCL's own streams take hardware queues as well: at 12
    # two of three lanes shared one queue and ran back to back (world-1 comm path 0.29 ms/frame, 0.22 at 16-24;
    # 1/8 shares 0.045 -> 0.043; profiles/r03_session2/comm_world1_hwq.jsonl)
    # library lanes (the default, below) are high-priority streams with hardware queues of their own: one GPU needs no
    # more than the default 4 (C2 0.180 ms/frame at 4 and at 12 queues, profiles/r05/lanes/)
    lib_lane_run = args.lanes == "library" and not classic and args.lane_priority is None
    # (a rank's share runs 8 lanes: more than the high-priority queues HIP hands out at 4, 0.046 against 0.038
    # ms/frame at 12-24 queues, profiles/r05/lanes/)
    want_q = 24 if (n > 1 or args.attach_comm) else (12 if share else (0 if (classic or lib_lane_run) else 12))
    if os.environ.get("RTAMD_HWQ"):                    # A/B studies: an explicit queue count
        os.environ["GPU_MAX_HW_QUEUES"] = os.environ["RTAMD_HWQ"]
    elif want_q and int(os.environ.get("GPU_MAX_HW_QUEUES", "4") or 4) < want_q:
        os.environ["GPU_MAX_HW_QUEUES"] = str(want_q)   # (the pool's boxes export 4, HIP's default)

    import numpy as np
    import torch
    import torch.distributed as dist
    from rtamd import Renderer, scenes

    torch.cuda.set_device(local_rank)
    if n > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))

    cfg = scenes.CONFIGS[args.config]
    assert FRAME_DIMS[args.config] == (cfg.width, cfg.height, cfg.spp), "FRAME_DIMS out of date"
    scene = scenes.config_scene(cfg)
    r = Renderer(scene, device=local_rank)
    for kv in args.pre_opt:
        k, v = kv.split("=")
        r.set_option(k, int(v, 0))
    if args.rebuild:                  # before the build: the build then leaves out the cold triangle records (auto)
        r.set_option("rebuild", 1)
    r.build_acceleration_structure(0, mode=args.build).configure_camera(cfg.width, cfg.height)
    r.set_option("kernel", args.kernel)
    for kv in args.opt:
        k, v = kv.split("=")
        r.set_option(k, int(v, 0))
    # measured: 4 lanes for a whole frame (3 with a per-frame rebuild), 8 lanes for a rank's 1/N
    # share (the library's auto grid then gives each launch 100 / lanes + 12 % of the GPU while others are in
    # flight: 37 % at 4 lanes, 24 % at 8; profiles/r03_session2/share_grid_*.txt, lanes_new*.txt)
    # a per-frame rebuild of a >= 16 M-path frame (C5): 2 lanes (the rebuild kernels then find slots between two
    # traces instead of three or four: 9.78 / 9.76 -> 8.82 ms/frame; 1 lane 13.7; profiles/r04/c5_rebuild/r04s17_*,
    # r04s18_*); trees built once keep 4 (5.46 against 5.86 with 3, 6.43 with 2)
    # library lanes (default): the scene picks the lanes ("overlap" -1, rt_api.cpp auto_lanes: the counts below) and
    # runs frames rendered without a stream on streams of its own; a C2-LBVH-style rebuild of a small frame ("classic")
    # keeps the caller's null stream as lane 0, which only a caller can hand it
    lib_lanes = args.lanes == "library" and not classic and args.lane_priority is None
    # (round 5: any per-frame rebuild, 2 — C5 1/8 share 5.5 -> 4.1 ms/frame, C2-LBVH 1.04 -> 0.38; profiles/r05/c5_rebuild/)
    L = max(1, args.overlap if args.overlap is not None else (2 if args.rebuild else (8 if share else 4)))
    overlap = L > 1
    if lib_lanes and args.overlap is None:
        r.set_option("overlap", -1)
    elif overlap:
        r.set_option("overlap", L)
    if share and not (lib_lanes and args.overlap is None):
        # the host stages frame k once frame k - depth's trace is done: 64 lets it run 8 frames ahead per lane
        # (C2 1/8 share 0.0446 -> 0.0432 ms/frame, C4 equal; profiles/r03_session2/stage_depth.jsonl)
        r.set_option("stage_depth", 64)
    info = r.info()
    stream = torch.cuda.current_stream().cuda_stream
    # "overlap": frame k runs on lanes[k % L]; each lane is a self-contained trace -> gather -> assemble chain
    lanes = [torch.cuda.current_stream()] + [torch.cuda.Stream() for _ in range(L - 1)] if overlap else None
    # every lane on a new stream, none on the null stream (C2 1/8 share 0.0437 -> 0.0416 ms/frame, world-1 comm
    # path 0.212 -> 0.191, the whole frame with 4 lanes above; profiles/r03_session2/lane_streams_*.txt)
    prio = args.lane_priority if args.lane_priority is not None else (None if classic else 0)
    if overlap and prio is not None and not lib_lanes:
        lanes = [torch.cuda.Stream(priority=prio) for _ in range(L)]
    shard = tuple(int(v) for v in args.shard.split("/")) if args.shard else None
    if shard and (n > 1 or args.attach_comm):
        raise SystemExit("--shard is a one-GPU study")

    tiles = None
    if n > 1 or args.attach_comm:
        # the library's multi-GPU frame (rt_scene_attach_comm): each rank traces its interleaved tiles,
        # the tiles are gathered to rank 0 over RCCL and assembled there, all on the frame's stream
        cid = [Renderer.comm_unique_id() if rank == 0 else None]
        if n > 1:
            dist.broadcast_object_list(cid, src=0)
        r.attach_comm(cid[0], rank, n, TILE, TILE)
    elif shard:
        tiles = (TILE, TILE, shard[0], shard[1])
    frame_buf = torch.zeros(cfg.width * cfg.height * 4, dtype=torch.uint8, device="cuda") if rank == 0 else None
    nbuf = rt_scene_lanes_max if overlap else 1
    serial_stream = torch.cuda.Stream()                    # the roofline's serialised launches (a non-null stream)
    frame_bufs = ([frame_buf] + [torch.zeros_like(frame_buf) if overlap else frame_buf for _ in range(nbuf - 1)]
                  if rank == 0 else [None] * nbuf)

    host_update = []                                       # (update_ms, part of it waiting on the GPU) per call

    def step(frame, sync=True, keep=False, one_stream=False, skip=False):
        """One frame; sync=False pipelines it (host TLAS build of the next frame overlaps the GPU).
        With "overlap", frame k runs on lanes[k % L] (its own trace -> gather -> assemble chain);
        one_stream: every frame on the first lane's stream (launches serialised back to back)."""
        b = frame % nbuf if overlap else 0
        if lib_lanes and overlap:
            st = serial_stream.cuda_stream if one_stream else None   # None: the scene's own lane streams
        else:
            st = lanes[0 if one_stream else frame % L].cuda_stream if overlap else stream
        fb = frame_bufs[b]
        t_call = time.perf_counter()
        _, _, sts = r.render(frame, exact=args.exact, want_rgba=False, rgba8_device=fb.data_ptr() if fb is not None else None,
                             stream=st, sync=sync, keep_counters=keep, tiles=tiles, skip_update=skip)
        host_update.append((sts["update_ms"], sts["update_wait_ms"], (time.perf_counter() - t_call) * 1e3))

    # clock warm-up: the GPU's clocks ramp up over the first ~0.1-0.5 s of load (measured: serialised C2 launches
    # 395 -> ~265 us, C3 2.8 -> 1.6 ms over the first launches, profiles/r03_*); a real-time renderer runs in
    # the steady state, so untimed frames are rendered for --clock-warmup seconds before the warm-up steps
    t_cw = time.perf_counter()
    k = 0
    # --overlap 1: every launch of the run is serialised, and the roofline is priced on all of them (the set a
    # rocprofv3 --stats average of this very command covers); the library's timing ring holds 256 launches
    pre_ms, pre_frames = [], []                            # ... with the frame each launch rendered
    while args.clock_warmup > 0:
        for _ in range(16):                                # chunks of 16 frames; ranks stop together (rank 0 decides)
            step(k % 1000, sync=False)
            pre_frames.append(k % 1000)
            k += 1
        torch.cuda.synchronize()
        pre_ms += list(r.collect()[1])
        done = torch.tensor([1.0 if time.perf_counter() - t_cw >= args.clock_warmup else 0.0], device="cuda")
        if n > 1:
            dist.broadcast(done, src=0)
        if done.item() > 0:
            break
    for f in range(args.warmup):                           # pipelined like the timed steps (and in the timing ring)
        step(f, sync=False)
        pre_frames.append(f)
    torch.cuda.synchronize()
    if n > 1:
        dist.barrier()
    torch.cuda.synchronize()

    pre_ms += list(r.collect()[1])                         # warm-up timings: not the timed region's
    host_update.clear()
    t0 = time.perf_counter()
    for k in range(args.steps):
        step(args.warmup + k, sync=False, keep=True, skip=args.skip_update)   # counters were zeroed by collect()
    torch.cuda.synchronize()
    if n > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    timed_update = np.asarray(host_update[:args.steps], dtype=np.float64).reshape(-1, 3)
    if args.launch_times and rank == 0:                    # before collect() empties the library's ring
        np.save(args.launch_times, r.debug_read("launch_times").view(np.float32).reshape(-1, 2))
    acc, kernel_ms = r.collect()                           # device counters + HIP-event kernel times
    if lib_lanes and args.overlap is None:
        L = int(r.info()["overlap_lanes"])                 # the library's pick for this frame kind
    rays = int(acc["rays"])
    assert len(kernel_ms) == args.steps, (len(kernel_ms), args.steps)

    # max over ranks of the elapsed time; total rays over ranks
    if n > 1:
        t = torch.tensor([elapsed, float(rays)], dtype=torch.float64, device="cuda")
        tmax = t.clone()
        dist.all_reduce(tmax[:1], op=dist.ReduceOp.MAX)
        dist.all_reduce(t[1:], op=dist.ReduceOp.SUM)
        elapsed, rays = float(tmax[0]), int(t[1])

    # the roofline's serialised launches: the timed frames again, back to back on one stream (no overlap partner,
    # so each launch has the whole GPU: "grid_pct" 100), the GPU kept busy so its clocks stay where the timed
    # region ran them; the HIP-event duration of each launch is the kernel's own
    if overlap:
        r.set_option("grid_pct", 100)
    for k in range(args.steps):
        step(args.warmup + k, sync=False, one_stream=True)
    torch.cuda.synchronize()
    _, serial_ms = r.collect()
    if overlap:
        r.set_option("grid_pct", 0)
    if n > 1:
        dist.barrier()
    # SURVEY 8d latency definition: wall time from the call to the framebuffer being ready (rank 0: the
    # assembled frame), synchronous frames, median of 20 after the timed region (untimed for `value`)
    lat = []
    n_lat = min(20, args.steps)
    for k in range(n_lat):                                 # the first timed frames, one at a time
        t1 = time.perf_counter()
        step(args.warmup + k, sync=False)                  # enqueue, then wait for the whole device
        torch.cuda.synchronize()
        lat.append((time.perf_counter() - t1) * 1e3)
    _, sync_ms = r.collect()
    if n > 1:
        dist.barrier()

    # untimed work-counting passes for the roofline: the animation changes a frame's work (C3's launches vary
    # 1.3-2.6 ms over the frames of one run), so every priced launch is priced with the work of the frame it
    # rendered — one counting pass per distinct frame (all ranks run the same passes: a pass gathers too)
    timed_frames = [args.warmup + k for k in range(args.steps)]
    serial_frames = list(timed_frames)                       # the serialised launches re-render the timed frames
    lat_frames = timed_frames[:n_lat]
    all_serial = not overlap                                 # every launch of the run was serialised
    priced_frames = (pre_frames + timed_frames + serial_frames + lat_frames) if all_serial else serial_frames
    assert not all_serial or len(priced_frames) == len(pre_ms) + len(kernel_ms) + len(serial_ms) + len(sync_ms), \
        (len(pre_frames), len(pre_ms), len(kernel_ms), len(serial_ms), len(sync_ms))
    work = {}
    torch.cuda.synchronize()
    for f in sorted(set(priced_frames + timed_frames)):
        _, _, work[f] = r.render(f, exact=args.exact, want_rgba=False, count_work=True,
                                 rgba8_device=frame_buf.data_ptr() if frame_buf is not None else None, tiles=tiles,
                                 stream=stream)
    if n > 1:
        dist.barrier()
    # the per-frame BLAS rebuild's own roofline (untimed; every rank rebuilds its replica, so rank 0's is the figure)
    rebuild_block = None
    if args.rebuild and not args.no_rebuild_roofline:
        torch.cuda.synchronize()
        r.synchronize()
        rebuild_block = rebuild_roofline(r, [args.warmup + args.steps + k for k in range(6)])
    if n > 1:
        dist.barrier()

    if rank == 0:
        avg_kernel_ms = float(np.mean(kernel_ms))            # timed region: launches overlap (L lanes)
        serial_kernel_ms = float(np.mean(serial_ms))         # the same kernel with no overlap partner, back to back
        sync_kernel_ms = float(np.mean(sync_ms))             # ... and after a host synchronisation each (latency frames)
        if all_serial:
            every = list(pre_ms) + list(kernel_ms) + list(serial_ms) + list(sync_ms)
            serial_kernel_ms = float(np.mean(every))
        # mean over the priced launches of their frames' counted work
        keys = ("rays", "pixels", "aabb_tests", "triangle_tests", "sphere_quad_tests", "quad_tests", "instance_visits", "hits")
        cst = {k: float(np.mean([work[f][k] for f in priced_frames])) for k in keys}
        bytes_launch = float(np.mean([algorithmic_bytes(work[f]) for f in priced_frames]))
        bytes_timed = float(np.mean([algorithmic_bytes(work[f]) for f in timed_frames]))
        achieved = bytes_launch / (serial_kernel_ms * 1e-3) / 1e9
        kname = ("render_persistent_kernel" if args.kernel else "render_kernel") + ("<exact>" if args.exact else "<fast>")
        tag = pmc_tag(args)
        traffic, traffic_src, traffic_why = load_traffic(tag)
        hbm_frac = traffic / (serial_kernel_ms * 1e-3) / (HBM_PEAK_GBS * 1e9) if traffic else None
        # what the counters say limits the kernel (null without a PMC summary of this exact workload)
        limiter = ("latency" if hbm_frac < LATENCY_BOUND_FRAC else "hbm") if hbm_frac is not None else None
        value = rays / elapsed / 1e6
        out = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "Mrays/s",
            "n_gpus": n,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed * 1e3 / args.steps, 4),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic",
            "config": {
                "workload": f"{cfg.name}: {cfg.description}",
                "width": cfg.width, "height": cfg.height, "spp": cfg.spp, "depth": cfg.depth,
                "triangles": scene.triangle_count, "instances": len(scene.instances),
                "blas_node_pairs": info["blas_node_pairs"],
                "parallelism": (f"screen-tiles{n} ({TILE}x{TILE} interleaved; rt_scene_attach_comm: RCCL gather + "
                                f"assemble inside rt_render, overlapped across {L} lanes)"
                                if n > 1 else (f"single-gpu, shard {args.shard} only" if shard else
                                               ("single-gpu through the world-1 comm path" if args.attach_comm
                                                else "single-gpu"))),
                "overlap_lanes": L,
                "lane_streams": (None if not overlap else
                                 ("the scene's own (overlap -1: lanes and staging picked by the library)"
                                  if lib_lanes and args.overlap is None else
                                  ("the scene's own" if lib_lanes else
                                   ("current stream + new streams" if prio is None else f"new streams, priority {prio}")))),
                "hw_queues": int(os.environ.get("GPU_MAX_HW_QUEUES", "4") or 4),
                "tile": TILE,
                "threshold": "auto (64 at depth x spp <= 2, else 40)",
                "options": args.pre_opt + args.opt,
                "kernel": ("EXACT" if args.exact else "FAST") + (" persistent" if args.kernel else " grid"),
                "bvh": args.build,
                "frames": "animated (Main.cu updateInstance), per-frame TLAS rebuild" +
                          (" on the GPU" if args.build == "lbvh" else " + upload") +
                          (", per-frame GPU BLAS rebuild" if args.rebuild else "") + ", pipelined",
            },
            "value_kind": (f"whole-frame throughput with {L} overlapped lanes (frame k+1's launch fills frame k's "
                           "tail); frame_latency_ms_median is the synchronous call-to-framebuffer time") if overlap
                          else "whole-frame throughput, serialised frames",
            "rays_per_frame": round(rays / args.steps, 1),
            "frame_latency_ms_median": round(float(np.median(lat)), 4),
            # SURVEY 8(d) as a rate: the latency frames' rays (counted) over the median synchronous call-to-framebuffer
            # time (one frame in flight, as the reference's loop keeps on its render stream, Renderer.cu:308-317)
            # (N > 1: rank 0 counted only its own tiles, so the timed frames' mean over all ranks is used)
            "value_latency": round((float(np.mean([work[f]["rays"] for f in lat_frames])) if n == 1 else rays / args.steps)
                                   / (float(np.median(lat)) * 1e-3) / 1e6, 2),
            "value_latency_unit": "Mrays/s",
            # host side of a timed rt_render call (update callback, instance records, TLAS build, staging)
            # and the part of it spent blocked on the GPU (a staging buffer still in use)
            "host_update_ms_median": round(float(np.median(timed_update[:, 0])), 4),
            "host_update_wait_ms_median": round(float(np.median(timed_update[:, 1])), 4),
            # the whole rt_render call of a timed (pipelined) frame on the host, its waits included: when it is
            # close to ms_per_step the frame rate is bound by the host's per-frame work, not by the GPU
            "host_call_ms_median": round(float(np.median(timed_update[:, 2])), 4),
            "host_busy_ms_median": round(float(np.median(timed_update[:, 2] - timed_update[:, 1])), 4),
            "host_call_ms_mean": round(float(np.mean(timed_update[:, 2])), 4),
            "host_update_wait_ms_mean": round(float(np.mean(timed_update[:, 1])), 4),
            "kernel_ms": round(serial_kernel_ms, 4),
            "kernel_ms_overlapped": round(avg_kernel_ms, 4),
            "kernel_ms_sync": round(sync_kernel_ms, 4),
            "clock_warmup_s": args.clock_warmup,
            "roofline": {
                "bound": "hbm",                                   # the roof `achieved` is priced against
                "limiter": limiter,
                "achieved": round(achieved, 2),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4),
                # the same bytes over the pipelined frame time (frames overlapped: ms_per_step), N = 1 only
                "frac_throughput": (round(bytes_timed / (elapsed / args.steps) / 1e9 / HBM_PEAK_GBS, 4)
                                    if n == 1 and not shard else None),
                "traffic": traffic,
                "traffic_source": traffic_src,
                "traffic_note": traffic_why,
                "lib_sha16": tag["lib_sha16"],
                "build": build_provenance(),
                "hbm_frac_measured": round(hbm_frac, 5) if hbm_frac is not None else None,
                "kernel": kname,
                "timing": (f"mean HIP-event duration of all {len(every)} launches of the run, every one serialised "
                           "(--overlap 1: the launches a rocprofv3 --stats average of this command covers; kernel_ms)"
                           if all_serial else
                           "mean HIP-event duration of the timed frames rendered again, serialised back to back on one "
                           "stream (kernel_ms)"),
                "bytes_formula": "SURVEY 8(d): 32 aabb + 36 tri + 32 sphere/quad + 48 inst + 32 ray + 4 pixel",
                "algorithmic_bytes_per_launch": int(bytes_launch),
                "layout_bytes_per_launch": int(layout_bytes(cst)),
                "work_per_launch": {k: int(round(cst[k])) for k in keys},
                "work_source": (f"RT_RENDER_COUNT_WORK pass of each priced launch's frame ({len(set(priced_frames))} "
                                f"distinct frames, mean over the {len(priced_frames)} priced launches)"),
            },
            "cpu_baseline": None,
        }
        if rebuild_block is not None:
            out["rebuild"] = rebuild_block
        if n == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(scene, cfg, args.cpu_seconds)
        print(json.dumps(out), flush=True)
    if n > 1:
        dist.barrier()
        dist.destroy_process_group()
    r.cleanup()


if __name__ == "__main__":
    main()
