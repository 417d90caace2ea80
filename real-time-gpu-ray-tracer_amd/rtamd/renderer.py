"""Python mirror of the reference's host `Renderer` (include/Global/Renderer.cuh:109-146) over
the C ABI of librtamd.so.  Method names follow the reference lifecycle:

    commitGeometryData + commitMaterialData + configureInstances -> Renderer(scene)
    buildAccelerationStructure                                   -> build_acceleration_structure()
    configureCamera                                              -> configure_camera()
    one iteration of startRender                                 -> render(frame)
    cleanup                                                      -> cleanup()

There is no CPU fallback: constructing a Renderer without librtamd.so or without a GPU raises.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import abi


class Renderer:
    def __init__(self, scene, device: int = 0, update=None):
        """update: None -> the scene's own animation (Main.cu updateInstance via the native
        rt_demo_update when scene.animated), False -> static, or a Python callable
        f(xforms: ctypes array of Xform, n, frame) (slow path, crosses into Python per frame)."""
        self.lib = abi.load_library()
        self.scene = scene
        self._cb = None
        if update is None:
            fn = C.cast(self.lib.rt_demo_update, C.c_void_p) if scene.animated else None
        elif update is False:
            fn = None
        else:
            self._cb = abi.UPDATE_FN(lambda user, xs, n, frame: update(xs, n, frame))
            fn = C.cast(self._cb, C.c_void_p)
        self._desc = scene.desc(fn)
        h = C.c_void_p()
        abi.check(self.lib, self.lib.rt_scene_create(C.byref(self._desc), device, C.byref(h)))
        self.h = h
        self.device = device
        self.width = self.height = 0

    # ---- lifecycle ---------------------------------------------------------------------
    def build_acceleration_structure(self, seed: int = 0, mode: str = "compat"):
        """mode "compat": the reference's random-axis median split (pinned seed); "sah": SAH trees;
        "lbvh": BLASes and the per-frame TLAS built on the GPU (linear BVH)."""
        m = {"compat": abi.RT_BUILD_COMPAT_MEDIAN, "sah": abi.RT_BUILD_SAH, "lbvh": abi.RT_BUILD_LBVH}[mode]
        abi.check(self.lib, self.lib.rt_scene_build(self.h, m, seed))
        return self

    def configure_camera(self, width: int, height: int, **camera):
        ci = self.scene.camera_input(**camera)
        abi.check(self.lib, self.lib.rt_camera_set(self.h, C.byref(ci), width, height))
        self.width, self.height = width, height
        self.camera = ci
        return self

    def set_camera(self, camera_input: abi.CameraInput):
        """Renderer::configureCamera with an explicit CameraInput (the interactive loop's moved camera,
        Renderer.cu:247-251 -> RenderPin.cu:73-95), same framebuffer size."""
        abi.check(self.lib, self.lib.rt_camera_set(self.h, C.byref(camera_input), self.width, self.height))
        self.camera = camera_input
        return self

    def set_comm_timeout(self, timeout_ms: int):
        """rt_comm_set_timeout: bounded waits on multi-GPU frames (0 = unbounded, async errors still polled)."""
        abi.check(self.lib, self.lib.rt_comm_set_timeout(self.h, int(timeout_ms)))
        return self

    def set_option(self, key: str, value: int):
        abi.check(self.lib, self.lib.rt_scene_set_option(self.h, key.encode(), int(value)))
        return self

    def update_triangles(self, first: int, triangles):
        """Replace triangles [first, first + len) (scenes.TRIANGLE_DTYPE array); "lbvh" scenes only."""
        t = np.ascontiguousarray(triangles)
        abi.check(self.lib, self.lib.rt_scene_update_triangles(self.h, first, t.shape[0], t.ctypes.data))
        return self

    def update_instances(self, first: int, instances):
        """Replace instance descriptions [first, first + len) (dicts as in scenes.Scene.instances)."""
        from .scenes import instance_desc_array
        arr = instance_desc_array(instances)
        abi.check(self.lib, self.lib.rt_scene_update_instances(self.h, first, len(instances), arr))
        return self

    def update(self, frame: int):
        abi.check(self.lib, self.lib.rt_scene_update(self.h, frame))

    def render(self, frame: int = 0, frame_seed: int = 0x5EED, exact: bool = False, count_work: bool = False,
               want_rgb: bool = False, want_rgba: bool = True, skip_update: bool = False,
               tiles=None, rgba8_device=None, rgb32_device=None, stream=None, sync: bool = True,
               keep_counters: bool = False):
        """One frame.  Returns (rgba[H,W,4] uint8 | None, rgb[H,W,3] float32 | None, stats dict).
        tiles = (tile_w, tile_h, rank, count) renders a tile shard into tile-compact outputs."""
        o = abi.RenderOpts()
        o.frame_seed = frame_seed
        o.flags = (abi.RT_RENDER_EXACT if exact else 0) | (abi.RT_RENDER_COUNT_WORK if count_work else 0) | \
                  (abi.RT_RENDER_SKIP_UPDATE if skip_update else 0) | (0 if sync else abi.RT_RENDER_NO_SYNC) | \
                  (abi.RT_RENDER_KEEP_COUNTERS if keep_counters else 0)
        comm = getattr(self, "comm", None)
        if comm is not None and comm[0] != 0:
            want_rgba = False                     # only rank 0 receives the assembled frame
        if tiles is not None:
            o.tile_w, o.tile_h, o.tile_rank, o.tile_count = tiles
            npix = self.tiles_for_rank(*tiles) * tiles[0] * tiles[1]
            shape = (npix,)
        else:
            shape = (self.height, self.width)
        o.rgba8_device = rgba8_device
        o.rgb32_device = rgb32_device
        o.stream = stream
        rgba = np.zeros(shape + (4,), np.uint8) if (want_rgba and sync) else None
        rgb = np.zeros(shape + (3,), np.float32) if (want_rgb and sync) else None
        st = abi.Stats()
        abi.check(self.lib, self.lib.rt_render(self.h, frame, C.byref(o),
                                               rgba.ctypes.data if rgba is not None else None,
                                               rgb.ctypes.data if rgb is not None else None, C.byref(st)))
        stats = {k: getattr(st, k) for k, _ in abi.Stats._fields_}
        return rgba, rgb, stats

    def collect(self, capacity: int = 256):
        """After pipelined renders: (accumulated stats dict, list of per-frame kernel ms)."""
        st = abi.Stats()
        ms = (C.c_float * capacity)()
        n = C.c_uint32()
        abi.check(self.lib, self.lib.rt_scene_collect(self.h, C.byref(st), ms, capacity, C.byref(n)))
        return {k: getattr(st, k) for k, _ in abi.Stats._fields_}, [ms[i] for i in range(n.value)]

    def debug_read(self, name: str) -> np.ndarray:
        """Debug buffer of the last launch that recorded it ("timeline", "costmap"), as raw bytes."""
        n = C.c_size_t()
        abi.check(self.lib, self.lib.rt_scene_debug_read(self.h, name.encode(), None, 0, C.byref(n)))
        buf = np.zeros(n.value, np.uint8)
        abi.check(self.lib, self.lib.rt_scene_debug_read(self.h, name.encode(), buf.ctypes.data, n.value, C.byref(n)))
        return buf

    def timeline(self):
        """Per-wave timeline of the last persistent launch (set_option("timeline", 1) first).
        Structured array: start/end in s_memrealtime ticks (100 MHz), xcc, hw_id, pixels."""
        w = self.debug_read("timeline").view(np.uint64).reshape(-1, 20)
        out = np.zeros(len(w), dtype=[("start", np.uint64), ("end", np.uint64), ("xcc", np.uint32),
                                      ("hw_id", np.uint32), ("pixels", np.uint32), ("exhaust", np.uint64),
                                      ("rounds", np.uint32), ("shades", np.uint32), ("grabs", np.uint32),
                                      ("cyc_refill", np.uint64), ("cyc_interior", np.uint64), ("cyc_leaf", np.uint64),
                                      ("cyc_shade", np.uint64), ("iters", np.uint64), ("refill_iters", np.uint64),
                                      ("cyc_lanes", np.uint64), ("cyc_scatter", np.uint64),
                                      ("lanes_interior", np.uint64), ("lanes_leaf_tlas", np.uint64),
                                      ("lanes_leaf_blas", np.uint64), ("lanes_shade", np.uint64)])
        out["start"], out["end"], out["exhaust"] = w[:, 0], w[:, 1], w[:, 4]
        out["xcc"], out["hw_id"], out["pixels"] = w[:, 2] & 0xFFFFFFFF, w[:, 2] >> 32, w[:, 3]
        out["rounds"], out["shades"], out["grabs"] = w[:, 5], w[:, 6], w[:, 7]
        out["cyc_refill"], out["cyc_interior"], out["cyc_leaf"], out["cyc_shade"] = w[:, 8], w[:, 9], w[:, 10], w[:, 11]
        out["iters"], out["refill_iters"] = w[:, 12], w[:, 13]
        out["cyc_lanes"], out["cyc_scatter"] = w[:, 14], w[:, 15]       # diagnostic builds only: lane refill work, scatter sampling
        # diagnostic builds only: lane sums per interior iteration / leaf phase (TLAS, BLAS leaves) / shade step
        out["lanes_interior"], out["lanes_leaf_tlas"], out["lanes_leaf_blas"], out["lanes_shade"] = w[:, 16], w[:, 17], w[:, 18], w[:, 19]
        return out

    def costmap(self):
        """Traversal rounds per output pixel of the last COUNT_WORK render with option "costmap"."""
        return self.debug_read("costmap").view(np.uint32)

    def tiles_for_rank(self, tile_w, tile_h, rank, count):
        return int(self.lib.rt_tiles_for_rank(self.h, tile_w, tile_h, rank, count))

    def assemble_tiles(self, gathered_device, slab_tiles, tile_w, tile_h, tile_count, frame_device, stream=None):
        abi.check(self.lib, self.lib.rt_assemble_tiles(self.h, gathered_device, slab_tiles, tile_w, tile_h,
                                                       tile_count, frame_device, stream))

    # ---- multi-GPU frames (rt_scene_attach_comm) ---------------------------------------------
    @staticmethod
    def comm_unique_id() -> bytes:
        """Rank 0: a fresh RCCL unique id (128 bytes) to hand to every rank out of band."""
        lib = abi.load_library()
        cid = abi.CommId()
        abi.check(lib, lib.rt_comm_unique_id(C.byref(cid)))
        return bytes(bytearray(cid))

    def attach_comm(self, comm_id: bytes, rank: int, world: int, tile_w: int = 64, tile_h: int = 64):
        """Make this scene rank `rank` of a `world`-GPU frame: render() traces this rank's tiles, gathers
        them to rank 0 over RCCL and assembles the frame there (collective over the ranks)."""
        cid = abi.CommId.from_buffer_copy(bytes(comm_id))
        abi.check(self.lib, self.lib.rt_scene_attach_comm(self.h, C.byref(cid), rank, world, tile_w, tile_h))
        self.comm = (rank, world, tile_w, tile_h)
        return self

    def detach_comm(self):
        abi.check(self.lib, self.lib.rt_scene_detach_comm(self.h))
        self.comm = None
        return self

    def trace_rays(self, rays, exact: bool = False):
        rays = np.ascontiguousarray(rays, np.float32).reshape(-1, 6)
        n = rays.shape[0]
        hits = (abi.Hit * max(1, n))()
        abi.check(self.lib, self.lib.rt_trace_rays(self.h, rays.ctypes.data, n,
                                                   abi.RT_RENDER_EXACT if exact else 0, hits))
        out = np.zeros(n, dtype=[("t", np.float32), ("instance", np.uint32), ("ptype", np.uint32),
                                 ("pindex", np.uint32), ("point", np.float32, 3), ("normal", np.float32, 3),
                                 ("mtype", np.uint32), ("midx", np.uint32)])
        out[:] = np.frombuffer(hits, dtype=out.dtype, count=n)
        return out

    def synchronize(self):
        abi.check(self.lib, self.lib.rt_synchronize(self.h))

    def info(self):
        i = abi.SceneInfo()
        abi.check(self.lib, self.lib.rt_scene_get_info(self.h, C.byref(i)))
        return {k: getattr(i, k) for k, _ in abi.SceneInfo._fields_}

    def export_blas(self, b: int):
        nn, npr = C.c_uint32(), C.c_uint32()
        abi.check(self.lib, self.lib.rt_scene_export_blas(self.h, b, None, None, None, C.byref(nn), C.byref(npr)))
        boxes = np.zeros((nn.value, 6), np.float32)
        ci = np.zeros((nn.value, 2), np.uint32)
        refs = np.zeros(npr.value, np.uint32)
        abi.check(self.lib, self.lib.rt_scene_export_blas(self.h, b, boxes.ctypes.data, ci.ctypes.data,
                                                          refs.ctypes.data, C.byref(nn), C.byref(npr)))
        return boxes, ci, refs

    def export_tlas(self):
        nn, npr = C.c_uint32(), C.c_uint32()
        abi.check(self.lib, self.lib.rt_scene_export_tlas(self.h, None, None, None, C.byref(nn), C.byref(npr)))
        boxes = np.zeros((nn.value, 6), np.float32)
        ci = np.zeros((nn.value, 2), np.uint32)
        refs = np.zeros(npr.value, np.uint32)
        abi.check(self.lib, self.lib.rt_scene_export_tlas(self.h, boxes.ctypes.data, ci.ctypes.data,
                                                          refs.ctypes.data, C.byref(nn), C.byref(npr)))
        return boxes, ci, refs

    def cleanup(self):
        if getattr(self, "h", None):
            self.lib.rt_scene_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.cleanup()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.cleanup()


BOX_MODES = {"reference": 0, "cull": 1, "decide": 2, "quad_pair": 3, "quad_greedy": 4}   # rt_box_mode (include/rt.h)


def box_test(boxes, rays, tmax=None, mode: str = "reference", device: int = 0):
    """rt_box_test: which boxes the trace kernel named by `mode` keeps for each (box, ray) in range [0.001, tmax]
    (tmax None = +inf); returns (hit bool array, entry t array, +inf on a miss)."""
    lib = abi.load_library()
    boxes = np.ascontiguousarray(boxes, np.float32).reshape(-1, 6)
    rays = np.ascontiguousarray(rays, np.float32).reshape(-1, 6)
    n = boxes.shape[0]
    if rays.shape[0] != n:
        raise ValueError("one ray per box")
    tm = np.full(n, np.inf, np.float32) if tmax is None else np.ascontiguousarray(
        np.broadcast_to(np.asarray(tmax, np.float32), (n,)))
    hit = np.zeros(max(1, n), np.uint8)
    te = np.zeros(max(1, n), np.float32)
    abi.check(lib, lib.rt_box_test(device, boxes.ctypes.data, rays.ctypes.data, tm.ctypes.data, n, BOX_MODES[mode],
                                   hit.ctypes.data, te.ctypes.data))
    return hit[:n].astype(bool), te[:n]
