#!/usr/bin/env python3
"""Serialised kernel time of a config at ray depth 1 (primary segments only) and at its own depth, to
split the launch into primary and secondary (bounce) work.

    python scripts/depth_probe.py [--config C2] [--frames 20] [--opt k=v]
"""
import argparse
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "real-time-gpu-ray-tracer_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C2")
    ap.add_argument("--frames", type=int, default=20)
    ap.add_argument("--opt", action="append", default=[])
    a = ap.parse_args()
    import torch
    from rtamd import Renderer, scenes
    torch.cuda.set_device(0)
    cfg = scenes.CONFIGS[a.config]
    scene = scenes.config_scene(cfg)
    fb = torch.zeros(cfg.width * cfg.height * 4, dtype=torch.uint8, device="cuda")
    for depth in sorted({1, cfg.depth}):
        r = Renderer(scene).build_acceleration_structure(0, mode="sah").configure_camera(
            cfg.width, cfg.height, ray_trace_depth=depth)
        for kv in a.opt:
            k, v = kv.split("=")
            r.set_option(k, int(v, 0))
        for f in range(10):
            r.render(f, want_rgba=False, rgba8_device=fb.data_ptr())
        ms, rays = [], 0
        for f in range(10, 10 + a.frames):
            _, _, st = r.render(f, want_rgba=False, rgba8_device=fb.data_ptr())
            ms.append(st["kernel_ms"])
            rays = st["rays"]
        print(json.dumps({"config": a.config, "depth": depth, "opts": a.opt, "kernel_ms_median": round(float(np.median(ms)), 4),
                          "rays_per_frame": rays}), flush=True)
        r.cleanup()


if __name__ == "__main__":
    main()
