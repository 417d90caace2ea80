#!/usr/bin/env python3
"""Traversal work per ray of one bench-configuration frame (RT_RENDER_COUNT_WORK): AABB tests (a quad visit = 4),
instance visits, primitive tests — to tell a slower library's extra work from extra instructions per step.
usage: [RTAMD_LIB=...] scripts/work_counts.py --config C2 [--build sah] [--opt k=v ...]; prints one JSON line."""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "real-time-gpu-ray-tracer_amd"))


def main():
    from rtamd import Renderer, scenes
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C2")
    ap.add_argument("--build", default="sah")
    ap.add_argument("--frames", default="0,37")
    ap.add_argument("--opt", action="append", default=[])
    ap.add_argument("--tag", default="")
    a = ap.parse_args()
    cfg = scenes.CONFIGS[a.config]
    r = Renderer(scenes.config_scene(cfg)).build_acceleration_structure(0, mode=a.build).configure_camera(cfg.width, cfg.height)
    for kv in a.opt:
        k, v = kv.split("=")
        r.set_option(k, int(v, 0))
    for f in (int(x) for x in a.frames.split(",")):
        _, _, st = r.render(f, count_work=True, want_rgba=False)
        rays = st["rays"]
        print(json.dumps({"tag": a.tag, "config": a.config, "frame": f, "rays": rays,
                          "aabb_per_ray": st["aabb_tests"] / rays, "inst_per_ray": st["instance_visits"] / rays,
                          "tri_per_ray": st["triangle_tests"] / rays, "sq_per_ray": st["sphere_quad_tests"] / rays,
                          "kernel_ms": st["kernel_ms"]}), flush=True)
    r.cleanup()


if __name__ == "__main__":
    main()
