#!/usr/bin/env python3
"""Kernel time vs workload shape (one process): which part of the path costs what."""
import json, os, statistics, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "real-time-gpu-ray-tracer_amd")]
import torch
from rtamd import Renderer, scenes

torch.cuda.set_device(0)
cases = [
    ("C2_d2", scenes.config_scene(scenes.CONFIGS["C2"]), dict()),
    ("C2_d1", scenes.config_scene(scenes.CONFIGS["C2"]), dict(ray_trace_depth=1)),
    ("demo_d2", scenes.demo_scene(), dict(ray_trace_depth=2, sample_count=1)),
    ("demo_d1", scenes.demo_scene(), dict(ray_trace_depth=1, sample_count=1)),
    ("C2_sky_d2", scenes.config_scene(scenes.CONFIGS["C2"]), dict(target=(0.0, 12.0, 0.0))),
    ("C2_down_d1", scenes.config_scene(scenes.CONFIGS["C2"]), dict(target=(0.0, -8.0, 0.0), ray_trace_depth=1)),
    ("C2_particles_d1", scenes.config_scene(scenes.CONFIGS["C2"]), dict(center=(0.0, 2.8, 4.0), target=(0.0, 2.8, 0.0), ray_trace_depth=1)),
]
fb = torch.zeros(1920 * 1080 * 4, dtype=torch.uint8, device="cuda")
for name, sc, cam in cases:
    r = Renderer(sc, update=False).build_acceleration_structure(0).configure_camera(1920, 1080, **cam)
    for kernel in (0, 1):
        r.set_option("kernel", kernel)
        _, _, cst = r.render(0, want_rgba=False, rgba8_device=fb.data_ptr(), count_work=True)
        ms = []
        for f in range(12):
            _, _, st = r.render(0, want_rgba=False, rgba8_device=fb.data_ptr())
            ms.append(st["kernel_ms"])
        med = statistics.median(ms[2:])
        rays = cst["rays"]
        print(json.dumps({"case": name, "kernel": ["grid", "persistent"][kernel], "kernel_ms": round(med, 4),
                          "rays": rays, "mrays_s": round(rays / med / 1e3, 1),
                          "pairs_per_ray": round(cst["aabb_tests"] / 2 / rays, 2),
                          "inst_per_ray": round(cst["instance_visits"] / rays, 2),
                          "tri_per_ray": round(cst["triangle_tests"] / rays, 2),
                          "sq_per_ray": round(cst["sphere_quad_tests"] / rays, 2),
                          "hit_frac": round(cst["hits"] / rays, 3),
                          "ns_per_ray": round(med * 1e6 / rays, 4)}), flush=True)
    r.cleanup()
