import sys, os
sys.path[:0]=[os.getcwd(), os.path.join(os.getcwd(),'real-time-gpu-ray-tracer_amd')]
import torch
from rtamd import Renderer, scenes
for c in ("C1","C2"):
    cfg=scenes.CONFIGS[c]
    for m in ("compat","sah"):
        r=Renderer(scenes.config_scene(cfg)).build_acceleration_structure(0, mode=m).configure_camera(cfg.width, cfg.height)
        r.render(0, want_rgba=False)
        print(c, m, r.info(), flush=True)
