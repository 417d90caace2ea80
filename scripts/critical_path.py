#!/usr/bin/env python3
"""How long does the heaviest pixel path take on its own?  (the floor of a serialised launch and of a rank's
1/N share: DESIGN.md §4-5)

    python scripts/critical_path.py [--config C2] [--build sah] [--opt k=v ...]

1. A COUNT_WORK frame with option "costmap" gives every pixel's traversal steps (interior steps + leaf phases).
2. The 8x8 units holding the heaviest, the median and a light pixel are traced alone (tile sharding with 8x8 tiles:
   rank = that unit's tile, count = all tiles), serialised, 30 launches each: the kernel time of a launch with one
   unit of work is that unit's critical path plus the launch's fixed cost (an empty-ish unit gives the latter).
3. The same for the heaviest unit with thresholds 1 and 64 (shade as soon as one lane / all lanes finished).
Prints one JSON line per measurement.
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
    ap.add_argument("--build", default="sah")
    ap.add_argument("--opt", action="append", default=[])
    ap.add_argument("--reps", type=int, default=30)
    a = ap.parse_args()
    import torch
    from rtamd import Renderer, scenes
    torch.cuda.set_device(0)
    cfg = scenes.CONFIGS[a.config]
    W, H = cfg.width, cfg.height
    r = Renderer(scenes.config_scene(cfg)).build_acceleration_structure(0, mode=a.build).configure_camera(W, H)
    for kv in a.opt:
        k, v = kv.split("=")
        r.set_option(k, int(v, 0))
    fb = torch.zeros(W * H * 4, dtype=torch.uint8, device="cuda")
    for f in range(3):
        r.render(f, want_rgba=False, rgba8_device=fb.data_ptr())
    r.set_option("costmap", 1)
    r.render(3, count_work=True, want_rgba=False, rgba8_device=fb.data_ptr())
    cm = r.costmap().reshape(H, W).astype(np.int64)
    r.set_option("costmap", 0)
    tx, ty = (W + 7) // 8, (H + 7) // 8
    ucm = np.zeros((ty * 8, tx * 8), np.int64)
    ucm[:H, :W] = cm
    units = ucm.reshape(ty, 8, tx, 8).transpose(0, 2, 1, 3).reshape(ty, tx, 64)
    umax = units.max(-1)
    order = np.argsort(umax.ravel())
    pick = {"heaviest": int(order[-1]), "p99": int(order[int(0.99 * len(order))]), "median": int(order[len(order) // 2]),
            "lightest": int(order[0])}
    print(json.dumps({"config": a.config, "pixel_steps_max": int(cm.max()), "pixel_steps_p999": float(np.percentile(cm, 99.9)),
                      "pixel_steps_mean": round(float(cm.mean()), 2), "units": int(umax.size)}), flush=True)
    count = tx * ty
    tbuf = torch.zeros(64 * 4, dtype=torch.uint8, device="cuda")

    def time_unit(u, thr=None):
        if thr is not None:
            r.set_option("threshold", thr)
        ms = []
        for k in range(a.reps):
            _, _, st = r.render(4, want_rgba=False, rgba8_device=tbuf.data_ptr(), tiles=(8, 8, u, count))
            ms.append(st["kernel_ms"])
        if thr is not None:
            r.set_option("threshold", 0)
        return float(np.median(ms)), float(np.min(ms))

    for name, u in pick.items():
        med, mn = time_unit(u)
        print(json.dumps({"unit": name, "unit_index": u, "max_steps": int(umax.ravel()[u]),
                          "sum_steps": int(units.reshape(-1, 64)[u].sum()), "kernel_ms_median": round(med, 4),
                          "kernel_ms_min": round(mn, 4)}), flush=True)
    for thr in (1, 8, 64):
        med, mn = time_unit(pick["heaviest"], thr)
        print(json.dumps({"unit": "heaviest", "threshold": thr, "kernel_ms_median": round(med, 4),
                          "kernel_ms_min": round(mn, 4)}), flush=True)
    r.cleanup()


if __name__ == "__main__":
    main()
