#!/usr/bin/env python3
"""Per-rank cost of the tile-sharded frame, emulated on one GPU (no RCCL).

    python scripts/shard_timing.py [--config C2] [--build sah] [--steps 20] [--counts 1 2 4 8]

For each rank count N it renders rank shares of the frame as bench.py's ranks do (64x64 tiles,
pipelined animated frames) and prints, per N: the slowest measured rank's mean kernel ms, that
rank's host-loop wall ms per frame, and the ideal strong-scaling kernel ms (N=1 kernel / N).
The gap is what an N-GPU frame loses before any gather cost.
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "real-time-gpu-ray-tracer_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C2")
    ap.add_argument("--build", default="sah")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--counts", type=int, nargs="+", default=[1, 2, 4, 8])
    ap.add_argument("--tile", type=int, default=64)
    ap.add_argument("--opt", action="append", default=[], help="scene option key=value")
    a = ap.parse_args()
    import numpy as np
    import torch
    from rtamd import Renderer, scenes
    torch.cuda.set_device(0)
    cfg = scenes.CONFIGS[a.config]
    r = Renderer(scenes.config_scene(cfg)).build_acceleration_structure(0, mode=a.build).configure_camera(
        cfg.width, cfg.height)
    for kv in a.opt:
        k, v = kv.split("=")
        r.set_option(k, int(v))
    stream = torch.cuda.current_stream().cuda_stream
    T = a.tile
    base = None
    for n in a.counts:
        worst = None
        for rank in (range(n) if n <= 4 else (0, 1)):     # ranks are alike; two suffice at N=8
            tiles = None if n == 1 else (T, T, rank, n)
            npx = cfg.width * cfg.height if n == 1 else r.tiles_for_rank(T, T, rank, n) * T * T
            buf = torch.zeros(npx * 4, dtype=torch.uint8, device="cuda")
            for f in range(a.warmup):
                r.render(f, want_rgba=False, tiles=tiles, rgba8_device=buf.data_ptr(), stream=stream)
            torch.cuda.synchronize()
            r.collect()
            t0 = time.perf_counter()
            for k in range(a.steps):
                r.render(a.warmup + k, want_rgba=False, tiles=tiles, rgba8_device=buf.data_ptr(), stream=stream,
                         sync=False, keep_counters=k > 0)
            torch.cuda.synchronize()
            wall = (time.perf_counter() - t0) * 1e3 / a.steps
            acc, kms = r.collect()
            _, _, st = r.render(a.warmup, want_rgba=False, tiles=tiles, rgba8_device=buf.data_ptr(), stream=stream)
            res = {"rank": rank, "kernel_ms": float(np.mean(kms)), "wall_ms": wall, "update_ms": st["update_ms"],
                   "rays": int(acc["rays"]) // a.steps, "pixels": npx}
            if worst is None or res["kernel_ms"] > worst["kernel_ms"]:
                worst = res
        if n == 1:
            base = worst["kernel_ms"]
        out = {"n": n, "slowest_rank": worst["rank"], "kernel_ms": round(worst["kernel_ms"], 4),
               "wall_ms_per_frame": round(worst["wall_ms"], 4), "host_update_ms": round(worst["update_ms"], 4),
               "rays": worst["rays"], "pixels": worst["pixels"]}
        if base:
            out["ideal_kernel_ms"] = round(base / n, 4)
            out["kernel_speedup"] = round(base / worst["kernel_ms"], 2)
        print(json.dumps(out), flush=True)
    r.cleanup()


if __name__ == "__main__":
    main()
