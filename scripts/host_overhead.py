#!/usr/bin/env python3
"""Host-side cost of one pipelined frame: wall time of the rt_render call (host instance update + TLAS
build + staging + launch submission, sync=False) and its update_ms, next to the GPU rate.

    python scripts/host_overhead.py [--config C2] [--shard R/N] [--lanes 3] [--frames 200] [--opt k=v]

If the per-call host time is close to bench.py's ms_per_step, the frame rate is host-bound.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "real-time-gpu-ray-tracer_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C2")
    ap.add_argument("--build", default="sah")
    ap.add_argument("--shard", default=None)
    ap.add_argument("--lanes", type=int, default=3)
    ap.add_argument("--frames", type=int, default=200)
    ap.add_argument("--opt", action="append", default=[])
    ap.add_argument("--pre-opt", action="append", default=[], help="option set before the build")
    a = ap.parse_args()
    import torch
    from rtamd import Renderer, scenes
    torch.cuda.set_device(0)
    cfg = scenes.CONFIGS[a.config]
    r = Renderer(scenes.config_scene(cfg))
    for kv in a.pre_opt:
        k, v = kv.split("=")
        r.set_option(k, int(v, 0))
    r.build_acceleration_structure(0, mode=a.build).configure_camera(cfg.width, cfg.height)
    for kv in a.opt:
        k, v = kv.split("=")
        r.set_option(k, int(v, 0))
    L = a.lanes
    if L > 1:
        r.set_option("overlap", L)
    lanes = [torch.cuda.current_stream()] + [torch.cuda.Stream() for _ in range(L - 1)]
    tiles = (64, 64) + tuple(int(v) for v in a.shard.split("/")) if a.shard else None
    fb = [torch.zeros(cfg.width * cfg.height * 4, dtype=torch.uint8, device="cuda") for _ in range(L)]

    def step(f):
        t = time.perf_counter()
        _, _, st = r.render(f, want_rgba=False, rgba8_device=fb[f % L].data_ptr(), stream=lanes[f % L].cuda_stream,
                            sync=False, keep_counters=True, tiles=tiles)
        return (time.perf_counter() - t) * 1e3, st["update_ms"], st["update_wait_ms"]

    for f in range(10):
        step(f)
    torch.cuda.synchronize()
    r.collect()
    calls, upd, wait = [], [], []
    t0 = time.perf_counter()
    for f in range(10, 10 + a.frames):
        c, u, w = step(f)
        calls.append(c)
        upd.append(u)
        wait.append(w)
    torch.cuda.synchronize()
    el = (time.perf_counter() - t0) * 1e3 / a.frames
    _, kms = r.collect(capacity=a.frames + 8)
    print(json.dumps({"config": a.config, "shard": a.shard, "lanes": L, "opts": a.pre_opt + a.opt, "ms_per_frame": round(el, 4),
                      "call_ms_p50_p90": [round(float(np.percentile(calls, q)), 4) for q in (50, 90)],
                      "update_ms_p50_p90": [round(float(np.percentile(upd, q)), 4) for q in (50, 90)],
                      "update_wait_ms_p50_p90": [round(float(np.percentile(wait, q)), 4) for q in (50, 90)],
                      "kernel_ms_mean": round(float(np.mean(kms)), 4) if kms else None}), flush=True)


if __name__ == "__main__":
    main()
