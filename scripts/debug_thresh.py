import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "real-time-gpu-ray-tracer_amd")]
import numpy as np, torch
from rtamd import Renderer, scenes
s = scenes.demo_with_particles(10)
r = Renderer(s).build_acceleration_structure(2).configure_camera(320, 180, ray_trace_depth=3, sample_count=4)
def go(kernel, thr, exact):
    r.set_option("kernel", kernel).set_option("threshold", thr)
    rgba, rgb, st = r.render(0, exact=exact, want_rgb=True, count_work=True)
    return rgb, st
for exact in (False, True):
    ref, rst = go(0, 16, exact)
    for thr in (1, 2, 4, 16, 64):
        for rep in range(3):
            rgb, st = go(1, thr, exact)
            d = (rgb != ref).any(axis=2)
            ys, xs = np.nonzero(d)
            print(f"exact={exact} thr={thr} rep={rep} ndiff={d.sum()} rays={st['rays']} vs {rst['rays']}",
                  list(zip(xs[:5].tolist(), ys[:5].tolist())), (rgb[ys[0], xs[0]], ref[ys[0], xs[0]]) if len(xs) else "")
