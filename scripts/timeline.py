#!/usr/bin/env python3
"""Per-wave timeline of the persistent render kernel (debug option "timeline").

    python scripts/timeline.py [--config C2] [--build sah] [--parts 8] [--out gpurun_out/timeline.npz]

Prints the launch span, how long waves live relative to it (a tail / ramp shows up as lifetime
fraction < 1), start/end spreads and per-XCD pixel shares and finish times.
"""
import argparse
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "real-time-gpu-ray-tracer_amd")]


def summarize(tl, tag):
    t0 = tl["start"].min()
    st = (tl["start"] - t0).astype(np.float64) * 0.01      # 100 MHz ticks -> us
    en = (tl["end"] - t0).astype(np.float64) * 0.01
    span = en.max()
    life = en - st
    per_xcc = {int(x): {"waves": int((tl["xcc"] == x).sum()), "pixels": int(tl["pixels"][tl["xcc"] == x].sum()),
                        "last_end_us": round(float(en[tl["xcc"] == x].max()), 1),
                        "median_end_us": round(float(np.median(en[tl["xcc"] == x])), 1)}
               for x in np.unique(tl["xcc"])}
    ex = (tl["exhaust"] - t0).astype(np.float64) * 0.01
    drain = en - ex
    return {"tag": tag, "waves": int(len(tl)), "span_us": round(float(span), 1),
            "exhaust_us_p1_p50_p99": [round(float(np.percentile(ex, q)), 1) for q in (1, 50, 99)],
            "drain_us_p50_p99_max": [round(float(np.percentile(drain, q)), 1) for q in (50, 99, 100)],
            "rounds_p50_max": [int(np.percentile(tl["rounds"], 50)), int(tl["rounds"].max())],
            "shades_p50_max": [int(np.percentile(tl["shades"], 50)), int(tl["shades"].max())],
            "grabs_p50": int(np.percentile(tl["grabs"], 50)),
            "cycle_split_refill_interior_leaf_shade": [round(float(tl[k].sum() / max(1, (tl["cyc_refill"] + tl["cyc_interior"] + tl["cyc_leaf"] + tl["cyc_shade"]).sum())), 3)
                                                        for k in ("cyc_refill", "cyc_interior", "cyc_leaf", "cyc_shade")],
            "stamped_cycles_over_life": round(float((tl["cyc_refill"] + tl["cyc_interior"] + tl["cyc_leaf"] + tl["cyc_shade"]).sum()
                                                    / max(1.0, ((tl["end"] - tl["start"]).astype(np.float64) * 0.01 * 1e-6).sum())) / 1e9, 3),
            "lanes_scatter_cycles_over_stamped": [round(float(tl[k].sum() / max(1, (tl["cyc_refill"] + tl["cyc_interior"] + tl["cyc_leaf"] + tl["cyc_shade"]).sum())), 3)
                                              for k in ("cyc_lanes", "cyc_scatter")],
            "cycles_per_interior_iter": round(float(tl["cyc_interior"].sum() / max(1, tl["iters"].sum())), 1),
            "interior_iters_per_round": round(float(tl["iters"].sum() / max(1, tl["rounds"].sum())), 2),
            "cycles_per_leaf_phase": round(float(tl["cyc_leaf"].sum() / max(1, tl["rounds"].sum())), 1),
            "cycles_per_shade": round(float(tl["cyc_shade"].sum() / max(1, tl["shades"].sum())), 1),
            "cycles_per_refill_iter": round(float(tl["cyc_refill"].sum() / max(1, tl["refill_iters"].sum())), 1),
            "refill_iters_per_shade": round(float(tl["refill_iters"].sum() / max(1, tl["shades"].sum())), 2),
            "us_per_round_plus_shade_p50": round(float(np.median(life / (tl["rounds"] + tl["shades"]))), 3),
            "mean_life_frac": round(float(life.mean() / span), 3),
            # diagnostic builds: mean lanes at work (of 64) per interior iteration, per leaf phase (TLAS + BLAS leaves,
            # which run as two divergent code paths) and per shade step
            "lanes_per_interior_iter": round(float(tl["lanes_interior"].sum() / max(1, tl["iters"].sum())), 2),
            "lanes_per_leaf_phase_tlas_blas": [round(float(tl["lanes_leaf_tlas"].sum() / max(1, tl["rounds"].sum())), 2),
                                               round(float(tl["lanes_leaf_blas"].sum() / max(1, tl["rounds"].sum())), 2)],
            "lanes_per_shade": round(float(tl["lanes_shade"].sum() / max(1, tl["shades"].sum())), 2),
            "start_us_p50_p99_max": [round(float(np.percentile(st, q)), 1) for q in (50, 99, 100)],
            "end_us_p1_p50_p99": [round(float(np.percentile(en, q)), 1) for q in (1, 50, 99)],
            "pixels": int(tl["pixels"].sum()), "per_xcc": per_xcc}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C2")
    ap.add_argument("--build", default="sah")
    ap.add_argument("--parts", type=int, nargs="+", default=[1, 8])
    ap.add_argument("--threshold", type=int, default=8)
    ap.add_argument("--out", default="gpurun_out/timeline.npz")
    ap.add_argument("--opt", action="append", default=[], help="extra scene option key=value")
    ap.add_argument("--pre-opt", action="append", default=[], help="scene option key=value set before the build")
    ap.add_argument("--shard", default=None, help="R/N: time rank R's 64x64-tile share of an N-rank split")
    a = ap.parse_args()
    tiles = (64, 64) + tuple(int(v) for v in a.shard.split("/")) if a.shard else None
    import torch
    from rtamd import Renderer, scenes
    torch.cuda.set_device(0)
    cfg = scenes.CONFIGS[a.config]
    fb = torch.zeros(cfg.width * cfg.height * 4, dtype=torch.uint8, device="cuda")
    r = Renderer(scenes.config_scene(cfg))
    for kv in a.pre_opt:
        k, v = kv.split("=")
        r.set_option(k, int(v))
    r.build_acceleration_structure(0, mode=a.build).configure_camera(cfg.width, cfg.height)
    r.set_option("threshold", a.threshold)
    for kv in a.opt:
        k, v = kv.split("=")
        r.set_option(k, int(v))
    saved = {}
    for parts in a.parts:
        r.set_option("queue_parts", parts)
        r.set_option("timeline", 0)
        for f in range(5):
            r.render(f, want_rgba=False, rgba8_device=fb.data_ptr(), tiles=tiles)
        r.set_option("timeline", 1)
        _, _, stt = r.render(5, want_rgba=False, rgba8_device=fb.data_ptr(), tiles=tiles)
        tl = r.timeline()
        saved[f"parts{parts}"] = tl
        s = summarize(tl, f"parts={parts}")
        s["kernel_ms_event"] = round(stt["kernel_ms"], 4)
        print(json.dumps(s), flush=True)
    r.set_option("timeline", 0)
    if tiles:
        np.savez(a.out, **saved)
        return
    # per-pixel traversal rounds (COUNT_WORK launch)
    r.set_option("costmap", 1)
    r.render(6, count_work=True, want_rgba=False, rgba8_device=fb.data_ptr())
    cm = r.costmap().reshape(cfg.height, cfg.width)
    r.set_option("costmap", 0)
    saved["costmap"] = cm
    units = cm[: cfg.height // 8 * 8].reshape(cfg.height // 8, 8, cfg.width // 8, 8).transpose(0, 2, 1, 3)
    ucost = units.reshape(units.shape[0], units.shape[1], 64)
    print(json.dumps({"costmap_rounds_pct_1_50_90_99_999_max": [float(np.percentile(cm, q)) for q in (1, 50, 90, 99, 99.9)]
                      + [int(cm.max())], "mean": round(float(cm.mean()), 2),
                      "unit_max_over_mean_pct_50_99": [round(float(np.percentile(ucost.max(-1) / np.maximum(1, ucost.mean(-1)), q)), 2)
                                                       for q in (50, 99)],
                      "unit_sum_pct_50_99_max": [float(np.percentile(ucost.sum(-1), q)) for q in (50, 99)] + [int(ucost.sum(-1).max())]}),
          flush=True)
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    np.savez(a.out, **saved)


if __name__ == "__main__":
    main()
