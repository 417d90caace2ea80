"""ctypes wrapper for liboracle.so — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module,
as the checker or the timed CPU baseline.  PARITY UNPINNED: see rt_oracle.h.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "liboracle.so")


def build(force: bool = False) -> str:
    if force or not os.path.exists(LIB) or \
            os.path.getmtime(LIB) < max(os.path.getmtime(os.path.join(HERE, f)) for f in ("rt_oracle.c", "rt_oracle.h")):
        subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB


class Counters(C.Structure):
    _fields_ = [("rays", C.c_uint64), ("aabb_tests", C.c_uint64), ("triangle_tests", C.c_uint64),
                ("sphere_quad_tests", C.c_uint64), ("instance_visits", C.c_uint64), ("node_pops", C.c_uint64)]

    def as_dict(self):
        return {k: int(getattr(self, k)) for k, _ in self._fields_}


_lib = None


def lib():
    global _lib
    if _lib is None:
        from rtamd import abi  # noqa: F401  (struct definitions shared with rt.h)
        L = C.CDLL(build())
        P = C.POINTER
        L.oracle_scene_create.argtypes = [P(abi.SceneDesc), C.c_uint64]
        L.oracle_scene_create.restype = C.c_void_p
        L.oracle_scene_destroy.argtypes = [C.c_void_p]
        L.oracle_scene_update.argtypes = [C.c_void_p, C.c_uint64]
        L.oracle_camera_set.argtypes = [C.c_void_p, P(abi.CameraInput), C.c_uint32, C.c_uint32]
        L.oracle_render.argtypes = [C.c_void_p, C.c_uint64, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32,
                                    C.c_void_p, C.c_void_p, C.c_int, C.c_int, P(Counters)]
        L.oracle_trace.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, P(abi.Hit), C.c_int, P(Counters)]
        for n in ("oracle_export_blas",):
            getattr(L, n).argtypes = [C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p, C.c_void_p,
                                      P(C.c_uint32), P(C.c_uint32)]
        L.oracle_export_tlas.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                         P(C.c_uint32), P(C.c_uint32)]
        L.oracle_blas_count.argtypes = [C.c_void_p]
        L.oracle_blas_count.restype = C.c_uint32
        for n in ("oracle_hit_sphere", "oracle_hit_parallelogram", "oracle_hit_triangle"):
            getattr(L, n).argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
        L.oracle_hit_aabb.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
        L.oracle_prim_bounds.argtypes = [C.c_uint32, C.c_void_p, C.c_void_p]
        L.oracle_prim_bounds.restype = None
        L.oracle_rng_init.argtypes = [C.c_uint64, C.c_uint64, C.c_uint64]
        L.oracle_rng_init.restype = C.c_uint64
        L.oracle_rng_uniform.argtypes = [P(C.c_uint64)]
        L.oracle_rng_uniform.restype = C.c_float
        L.oracle_instance_matrices.argtypes = [P(abi.Xform), C.c_void_p]
        L.oracle_instance_matrices.restype = None
        L.oracle_camera_export.argtypes = [C.c_void_p, C.c_void_p]
        L.oracle_instance_state.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p]
        L.oracle_demo_update.argtypes = [C.c_void_p, P(abi.Xform), C.c_size_t, C.c_uint64]
        L.oracle_demo_update.restype = None
        _lib = L
    return _lib


def _f32(a):
    return np.ascontiguousarray(a, dtype=np.float32)


class OracleScene:
    """CPU reference scene: build -> update(frame) -> camera -> render / trace."""

    def __init__(self, scene, build_seed: int = 0):
        from rtamd import abi
        L = lib()
        fn = C.cast(L.oracle_demo_update, C.c_void_p) if scene.animated else None
        desc = scene.desc(fn)
        self._scene = scene
        self.h = L.oracle_scene_create(C.byref(desc), build_seed)
        if not self.h:
            raise ValueError("oracle_scene_create failed (invalid scene)")
        self.width = self.height = 0
        self._abi = abi

    def close(self):
        if self.h:
            lib().oracle_scene_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def update(self, frame: int):
        assert lib().oracle_scene_update(self.h, frame) == 0

    def camera(self, width: int, height: int, **over):
        ci = self._scene.camera_input(**over)
        assert lib().oracle_camera_set(self.h, C.byref(ci), width, height) == 0
        self.width, self.height = width, height

    def camera_export(self):
        out = np.zeros(20, np.float32)
        assert lib().oracle_camera_export(self.h, out.ctypes.data) == 0
        return out

    def render(self, frame_seed: int = 0x5EED, region=None, threads: int = 1, brute_force: bool = False,
               want_rgb: bool = True, want_rgba: bool = True):
        x0, y0, w, h = region if region is not None else (0, 0, self.width, self.height)
        rgb = np.zeros((h, w, 3), np.float32) if want_rgb else None
        rgba = np.zeros((h, w, 4), np.uint8) if want_rgba else None
        cnt = Counters()
        rc = lib().oracle_render(self.h, frame_seed, x0, y0, w, h,
                                 rgb.ctypes.data if rgb is not None else None,
                                 rgba.ctypes.data if rgba is not None else None,
                                 int(threads), int(brute_force), C.byref(cnt))
        assert rc == 0, rc
        return rgb, rgba, cnt.as_dict()

    def trace(self, rays, brute_force: bool = False):
        rays = _f32(rays).reshape(-1, 6)
        n = rays.shape[0]
        hits = (self._abi.Hit * max(1, n))()
        cnt = Counters()
        assert lib().oracle_trace(self.h, rays.ctypes.data, n, hits, int(brute_force), C.byref(cnt)) == 0
        return hits_to_numpy(hits, n), cnt.as_dict()

    def instance_state(self):
        """(n_inst, 45) float32: inverse / forward / inverse-transpose rows 1-3, transformed box, centroid."""
        n = len(self._scene.instances)
        out = np.zeros((n, 45), np.float32)
        for i in range(n):
            assert lib().oracle_instance_state(self.h, i, out[i].ctypes.data) == 0
        return out

    def blas_count(self):
        return lib().oracle_blas_count(self.h)

    def export_blas(self, b: int):
        nn, npr = C.c_uint32(), C.c_uint32()
        assert lib().oracle_export_blas(self.h, b, None, None, None, C.byref(nn), C.byref(npr)) == 0
        boxes = np.zeros((nn.value, 6), np.float32)
        ci = np.zeros((nn.value, 2), np.uint32)
        refs = np.zeros(npr.value, np.uint32)
        assert lib().oracle_export_blas(self.h, b, boxes.ctypes.data, ci.ctypes.data, refs.ctypes.data,
                                        C.byref(nn), C.byref(npr)) == 0
        return boxes, ci, refs

    def export_tlas(self):
        nn, npr = C.c_uint32(), C.c_uint32()
        assert lib().oracle_export_tlas(self.h, None, None, None, C.byref(nn), C.byref(npr)) == 0
        boxes = np.zeros((nn.value, 6), np.float32)
        ci = np.zeros((nn.value, 2), np.uint32)
        refs = np.zeros(npr.value, np.uint32)
        assert lib().oracle_export_tlas(self.h, boxes.ctypes.data, ci.ctypes.data, refs.ctypes.data,
                                        C.byref(nn), C.byref(npr)) == 0
        return boxes, ci, refs


def hits_to_numpy(hits, n):
    out = np.zeros(n, dtype=[("t", np.float32), ("instance", np.uint32), ("ptype", np.uint32),
                             ("pindex", np.uint32), ("point", np.float32, 3), ("normal", np.float32, 3),
                             ("mtype", np.uint32), ("midx", np.uint32)])
    raw = np.frombuffer(hits, dtype=out.dtype, count=n)
    out[:] = raw
    return out


def rng_stream(seed: int, sub: int, n: int):
    st = C.c_uint64(lib().oracle_rng_init(seed, sub, 0))
    return np.array([lib().oracle_rng_uniform(C.byref(st)) for _ in range(n)], np.float32)
