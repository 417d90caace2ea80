#!/usr/bin/env python3
"""Generate tests/golden/*.npz from the oracle (oracle/rt_oracle.c).

The reference cannot be built or run here and holds no fixtures of its own, so
these vectors are produced by the oracle — the line-by-line restatement — and freeze it:
tests/test_golden.py re-derives them on CPU, tests/test_gpu_golden.py checks the HIP path
against them.  Regenerate only on an intentional oracle change:  python tests/golden/make_golden.py
"""
import ctypes as C
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [REPO, os.path.join(REPO, "real-time-gpu-ray-tracer_amd")]

from oracle.oracle import OracleScene, lib  # noqa: E402
from rtamd import abi, scenes  # noqa: E402


def prim_kats(seed=1234, n=4096):
    """(1) Seeded rays against one primitive of each type -> hit flag + 9 outputs."""
    g = np.random.default_rng(seed)
    prims = {
        "sphere": abi.Sphere(abi.Vec3(0.3, -0.2, 0.1), 1.3, 0, 0),
        "quad": abi.Parallelogram(abi.Vec3(-1, -0.5, 0.2), abi.Vec3(2, 0.3, 0), abi.Vec3(0.2, 1.7, 0.4), 0, 0),
        "tri": None,
    }
    t = abi.Triangle()
    for i, v in enumerate(((-1, -1, 0.1), (1.2, -0.8, -0.2), (0.1, 1.1, 0.3))):
        t.vertex[i] = abi.Vec3(*v)
    for i, v in enumerate(((0, 0, 1), (0.3, 0, 0.95), (0, 0.3, 0.95))):
        t.normal[i] = abi.Vec3(*v)
    t.has_normals = 1
    prims["tri"] = t
    fns = {"sphere": lib().oracle_hit_sphere, "quad": lib().oracle_hit_parallelogram, "tri": lib().oracle_hit_triangle}
    out = {}
    aim = {"sphere": ((0.3, -0.2, 0.1), 1.6), "quad": ((0.1, 0.5, 0.4), 1.4), "tri": ((0.1, -0.2, 0.1), 1.1)}
    for k, p in prims.items():
        o = g.uniform(-3, 3, (n, 3))
        o[:, 2] = g.uniform(2.5, 5, n)
        c, ext = aim[k]
        tgt = np.asarray(c) + g.uniform(-ext, ext, (n, 3))     # aimed near the primitive: ~half hit
        d = tgt - o
        d *= g.uniform(0.5, 2.0, (n, 1)) / np.linalg.norm(d, axis=1, keepdims=True)   # unnormalised too
        rays = np.concatenate([o, d], 1).astype(np.float32)
        rng = np.asarray([0.001, np.inf], np.float32)
        res = np.zeros((n, 10), np.float32)
        for i in range(n):
            r = np.zeros(9, np.float32)
            res[i, 0] = fns[k](C.byref(p), rays[i].ctypes.data, rng.ctypes.data, r.ctypes.data)
            res[i, 1:] = r
        out[f"{k}_rays"] = rays
        out[f"{k}_out"] = res
    boxes = g.uniform(-2, 2, (n, 3))
    ext = g.uniform(0.0, 1.5, (n, 3))
    b6 = np.stack([boxes[:, 0], boxes[:, 0] + ext[:, 0], boxes[:, 1], boxes[:, 1] + ext[:, 1],
                   boxes[:, 2], boxes[:, 2] + ext[:, 2]], 1).astype(np.float32)
    o = g.uniform(-4, 4, (n, 3))
    centre = boxes + ext / 2
    d = (centre - o) + g.normal(size=(n, 3)) * 0.8      # aimed at the box: roughly half hit
    d[g.random(n) < 0.1, 0] = 0.0                      # parallel-axis branch
    rays = np.concatenate([o, d], 1).astype(np.float32)
    res = np.zeros((n, 2), np.float32)
    rng = np.asarray([0.001, np.inf], np.float32)
    for i in range(n):
        te = np.zeros(1, np.float32)
        res[i, 0] = lib().oracle_hit_aabb(b6[i].ctypes.data, rays[i].ctypes.data, rng.ctypes.data, te.ctypes.data)
        res[i, 1] = te[0]
    out["aabb_boxes"], out["aabb_rays"], out["aabb_out"] = b6, rays, res
    return out


def grid_rays(o, width=64, height=36):
    """Primary rays through pixel centres (Kernel.cu:119-135 without jitter)."""
    c = o.camera_export()
    po, dx, dy, center = c[0:3], c[3:6], c[6:9], c[9:12]
    rays = []
    for y in range(height):
        for x in range(width):
            sp = (po + dx * np.float32(x)) + dy * np.float32(y)
            d = sp - center
            d = d / np.sqrt(np.float32((d * d).sum()))
            rays.append(np.concatenate([center, d]))
    return np.asarray(rays, np.float32)


def hits_and_images():
    out = {}
    s = scenes.demo_with_particles(12)
    o = OracleScene(s, build_seed=5)
    o.camera(64, 36)
    rays = grid_rays(o)
    h, _ = o.trace(rays)
    out["grid_rays"] = rays
    for k in h.dtype.names:
        out[f"grid_{k}"] = h[k]
    # BVH dumps: BLAS of the first particle, TLAS at frame 0
    nb = o.blas_count()
    b = o.export_blas(nb - 1)
    out["blas_boxes"], out["blas_ci"], out["blas_refs"] = b
    t = o.export_tlas()
    out["tlas_boxes"], out["tlas_ci"], out["tlas_refs"] = t
    # float RGB crops
    imgs = {}
    for name, scn, cam, frame in (
            ("demo_d1", scenes.demo_scene(), dict(ray_trace_depth=1), 0),
            ("demo_d2", scenes.demo_scene(), dict(ray_trace_depth=2), 0),
            ("demo_d10", scenes.demo_scene(), dict(ray_trace_depth=10), 0),
            ("demo_d10_f37", scenes.demo_scene(), dict(ray_trace_depth=10), 37),
            ("demo_spp4_d4", scenes.demo_scene(), dict(ray_trace_depth=4, sample_count=4), 0),
            ("particles_d2", scenes.demo_with_particles(12), dict(ray_trace_depth=2), 0)):
        o = OracleScene(scn, build_seed=5)
        o.camera(240, 160, **cam)
        if frame:
            o.update(frame)
        rgb, rgba, cnt = o.render(region=(72, 48, 96, 64), threads=8)
        imgs[name] = (rgb, rgba, cnt["rays"])
    for name, (rgb, rgba, rays) in imgs.items():
        out[f"img_{name}_rgb"] = rgb
        out[f"img_{name}_rgba"] = rgba
        out[f"img_{name}_rays"] = np.asarray(rays, np.int64)
    return out


def main():
    np.savez_compressed(os.path.join(HERE, "prim_kats.npz"), **prim_kats())
    np.savez_compressed(os.path.join(HERE, "scene_vectors.npz"), **hits_and_images())
    print("written", os.listdir(HERE))


if __name__ == "__main__":
    main()
