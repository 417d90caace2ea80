#!/usr/bin/env python3
"""GPU-built BLASes with and without TriCold records (option "cold_records") render the same frames: float RGB
bit for bit, FAST and EXACT, frames 0 and 37 (C2 with an instance group, C5)."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "real-time-gpu-ray-tracer_amd"))
from rtamd import Renderer, scenes  # noqa: E402


def main():
    for name in sys.argv[1:] or ["C2", "C5"]:
        cfg = scenes.CONFIGS[name]
        scene = scenes.config_scene(cfg)
        out = {}
        for cold in (0, 1):
            r = Renderer(scene).set_option("cold_records", cold).build_acceleration_structure(0, mode="lbvh")
            r.configure_camera(cfg.width, cfg.height, sample_count=cfg.spp, ray_trace_depth=cfg.depth)
            r.set_option("rebuild", 1)
            out[cold] = [r.render(f, want_rgb=True, exact=ex)[1] for f in (0, 37) for ex in (False, True)]
            r.cleanup()
        same = [bool(np.array_equal(a, b)) for a, b in zip(out[0], out[1])]
        print(name, "identical (f0 fast, f0 exact, f37 fast, f37 exact):", same, flush=True)
        assert all(same)


if __name__ == "__main__":
    main()
