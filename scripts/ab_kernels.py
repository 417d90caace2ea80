#!/usr/bin/env python3
"""A/B kernel variants in ONE process, interleaved rounds (cdna_hip_programming.md §5.4 rule 24).

    python scripts/ab_kernels.py [--config C2] [--rounds 5] [--frames 10] VARIANT ...
VARIANT = name:key=value,key=value  (keys: kernel, threshold; exact=1 selects the EXACT kernel)
Prints per-variant median / min kernel ms and Mrays/s (kernel-time based) as JSON lines.
"""
import argparse
import json
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "real-time-gpu-ray-tracer_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C2")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--frames", type=int, default=10)
    ap.add_argument("variants", nargs="+")
    a = ap.parse_args()
    import torch
    from rtamd import Renderer, scenes
    torch.cuda.set_device(0)
    cfg = scenes.CONFIGS[a.config]
    fb = torch.zeros(cfg.width * cfg.height * 4, dtype=torch.uint8, device="cuda")
    variants = []
    for v in a.variants:
        name, _, kv = v.partition(":")
        opts = dict(x.split("=") for x in kv.split(",") if x)
        variants.append((name, {k: (x if k == "build" else int(x)) for k, x in opts.items()}))
    renderers = {}

    def rkey(opts):      # one renderer per build mode and set of pre-build options ("pre_<key>=v")
        return (opts.get("build", "compat"),) + tuple(sorted((k, v) for k, v in opts.items() if k.startswith("pre_")))

    for _, opts in variants:
        key = rkey(opts)
        if key not in renderers:
            r = Renderer(scenes.config_scene(cfg))
            for k, v in key[1:]:
                r.set_option(k[4:], v)
            renderers[key] = r.build_acceleration_structure(0, mode=key[0]).configure_camera(cfg.width, cfg.height)
    res = {n: [] for n, _ in variants}
    rays = {}
    for rnd in range(a.rounds + 1):
        for name, opts in variants:
            exact = bool(opts.get("exact", 0))
            r = renderers[rkey(opts)]
            for k, x in opts.items():
                if k not in ("exact", "build") and not k.startswith("pre_"):
                    r.set_option(k, x)
            for f in range(a.frames):
                _, _, st = r.render(f, exact=exact, want_rgba=False, rgba8_device=fb.data_ptr())
                if rnd > 0:
                    res[name].append(st["kernel_ms"])
                rays[name] = st["rays"]
    for name, _ in variants:
        ms = res[name]
        med = statistics.median(ms)
        print(json.dumps({"variant": name, "median_kernel_ms": round(med, 4), "min_kernel_ms": round(min(ms), 4),
                          "mrays_per_s_kernel": round(rays[name] / med / 1e3, 1), "rays": rays[name], "n": len(ms)}),
              flush=True)


if __name__ == "__main__":
    main()
