#!/usr/bin/env python3
"""Per-frame GPU BLAS rebuild cost alone (no trace): rt_scene_update with option "rebuild" on an LBVH scene.
Prints one JSON line {config, updates, ms_per_update}.  Run under rocprofv3 --kernel-trace --stats for the
per-kernel breakdown of a rebuild that shares the GPU with nothing."""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "real-time-gpu-ray-tracer_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C5")
    ap.add_argument("--updates", type=int, default=20)
    ap.add_argument("--opt", action="append", default=[])
    ap.add_argument("--pre-opt", action="append", default=[], help="options set before the build")
    a = ap.parse_args()
    from rtamd import Renderer, scenes
    cfg = scenes.CONFIGS[a.config]
    r = Renderer(scenes.config_scene(cfg))
    for kv in a.pre_opt:
        k, v = kv.split("=")
        r.set_option(k, int(v))
    r.set_option("rebuild", 1)                           # before the build (no cold records, as bench.py)
    r.build_acceleration_structure(0, mode="lbvh")
    r.configure_camera(cfg.width, cfg.height, sample_count=cfg.spp, ray_trace_depth=cfg.depth)
    for kv in a.opt:
        k, v = kv.split("=")
        r.set_option(k, int(v))
    r.render(0)
    for f in range(1, 4):
        r.update(f)
    r.synchronize()
    t0 = time.perf_counter()
    for f in range(4, 4 + a.updates):
        r.update(f)
    r.synchronize()
    ms = (time.perf_counter() - t0) / a.updates * 1e3
    print(json.dumps({"config": a.config, "updates": a.updates, "ms_per_update": round(ms, 4), "opts": a.pre_opt + a.opt}), flush=True)
    r.cleanup()


if __name__ == "__main__":
    main()
