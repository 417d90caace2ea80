"""ctypes mirror of include/rt.h (the C ABI of librtamd.so).

Struct layouts here must match include/rt.h field for field; tests/test_abi.py checks the
sizes against the compiled library's view (rt_abi_version + sizeof probes via offsets).
"""
from __future__ import annotations

import ctypes as C
import os

RT_ABI_VERSION = 3

RT_OK = 0
RT_STATUS_NAMES = {
    0: "RT_OK", 1: "RT_ERR_INVALID_ARGUMENT", 2: "RT_ERR_DEVICE", 3: "RT_ERR_OUT_OF_MEMORY",
    4: "RT_ERR_STATE", 5: "RT_ERR_UNSUPPORTED",
}

# include/Basic/BasicTypes.cuh:9-16
SPHERE, PARALLELOGRAM, TRIANGLE = 0, 1, 2
ROUGH, METAL = 0, 1

RT_BUILD_COMPAT_MEDIAN = 0
RT_BUILD_SAH = 1
RT_BUILD_LBVH = 2

RT_RENDER_EXACT = 1 << 0
RT_RENDER_COUNT_WORK = 1 << 1
RT_RENDER_NO_SYNC = 1 << 2
RT_RENDER_SKIP_UPDATE = 1 << 3
RT_RENDER_KEEP_COUNTERS = 1 << 4

MISS = 0xFFFFFFFF


class Vec3(C.Structure):
    _fields_ = [("x", C.c_float), ("y", C.c_float), ("z", C.c_float)]

    @classmethod
    def of(cls, v):
        return cls(float(v[0]), float(v[1]), float(v[2]))

    def tuple(self):
        return (self.x, self.y, self.z)


class Sphere(C.Structure):
    _fields_ = [("center", Vec3), ("radius", C.c_float),
                ("material_type", C.c_uint32), ("material_index", C.c_uint32)]


class Parallelogram(C.Structure):
    _fields_ = [("q", Vec3), ("u", Vec3), ("v", Vec3),
                ("material_type", C.c_uint32), ("material_index", C.c_uint32)]


class Triangle(C.Structure):
    _fields_ = [("vertex", Vec3 * 3), ("normal", Vec3 * 3),
                ("material_type", C.c_uint32), ("material_index", C.c_uint32),
                ("has_normals", C.c_uint32), ("reserved", C.c_uint32)]


class Rough(C.Structure):
    _fields_ = [("albedo", Vec3)]


class Metal(C.Structure):
    _fields_ = [("albedo", Vec3), ("fuzz", C.c_float)]


class Xform(C.Structure):
    _fields_ = [("shift", Vec3), ("rotate_deg", Vec3), ("scale", Vec3)]


class InstanceDesc(C.Structure):
    _fields_ = [("primitive_type", C.c_uint32), ("primitive_index", C.c_uint32),
                ("primitive_count", C.c_uint32), ("has_local_bounds", C.c_uint32),
                ("local_bounds", C.c_float * 6), ("local_centroid", Vec3),
                ("xform", Xform)]


UPDATE_FN = C.CFUNCTYPE(None, C.c_void_p, C.POINTER(Xform), C.c_size_t, C.c_uint64)


class SceneDesc(C.Structure):
    _fields_ = [("spheres", C.POINTER(Sphere)), ("sphere_count", C.c_size_t),
                ("parallelograms", C.POINTER(Parallelogram)), ("parallelogram_count", C.c_size_t),
                ("triangles", C.POINTER(Triangle)), ("triangle_count", C.c_size_t),
                ("roughs", C.POINTER(Rough)), ("rough_count", C.c_size_t),
                ("metals", C.POINTER(Metal)), ("metal_count", C.c_size_t),
                ("instances", C.POINTER(InstanceDesc)), ("instance_count", C.c_size_t),
                ("update", C.c_void_p), ("update_user", C.c_void_p)]


class CameraInput(C.Structure):
    _fields_ = [("background", Vec3), ("center", Vec3), ("target", Vec3), ("fov", C.c_float),
                ("up", Vec3), ("focus_disk_radius", C.c_float), ("sample_range", C.c_float),
                ("sample_count", C.c_uint32), ("ray_trace_depth", C.c_uint32)]


class RenderOpts(C.Structure):
    _fields_ = [("frame_seed", C.c_uint64), ("flags", C.c_uint32),
                ("tile_w", C.c_uint32), ("tile_h", C.c_uint32),
                ("tile_rank", C.c_uint32), ("tile_count", C.c_uint32),
                ("rgba8_device", C.c_void_p), ("rgb32_device", C.c_void_p), ("stream", C.c_void_p)]


class Stats(C.Structure):
    _fields_ = [("rays", C.c_uint64), ("pixels", C.c_uint64), ("aabb_tests", C.c_uint64),
                ("triangle_tests", C.c_uint64), ("sphere_quad_tests", C.c_uint64),
                ("quad_tests", C.c_uint64), ("instance_visits", C.c_uint64), ("hits", C.c_uint64),
                ("kernel_ms", C.c_double),
                ("frame_ms", C.c_double), ("update_ms", C.c_double), ("update_wait_ms", C.c_double)]


class Hit(C.Structure):
    _fields_ = [("t", C.c_float), ("instance", C.c_uint32), ("primitive_type", C.c_uint32),
                ("primitive_index", C.c_uint32), ("point", Vec3), ("normal", Vec3),
                ("material_type", C.c_uint32), ("material_index", C.c_uint32)]


class SceneInfo(C.Structure):
    _fields_ = [("blas_count", C.c_uint64), ("blas_node_pairs", C.c_uint64),
                ("blas_leaves", C.c_uint64), ("tlas_node_pairs", C.c_uint64),
                ("device_bytes", C.c_uint64), ("width", C.c_uint32), ("height", C.c_uint32),
                ("sqrt_sample_count", C.c_uint32), ("ray_trace_depth", C.c_uint32),
                ("tlas_height", C.c_uint32), ("blas_height_max", C.c_uint32), ("overlap_lanes", C.c_uint32),
                ("stage_depth", C.c_uint32)]


class CommId(C.Structure):
    """rt_comm_id (= ncclUniqueId, 128 opaque bytes)."""
    _fields_ = [("internal", C.c_char * 128)]


class CameraControl(C.Structure):
    """rt_camera_control: OperateArgs (SDL_OpenGLWindow.cuh:34-45) + the loop's relative-mouse state."""
    _fields_ = [("mouse_sensitivity", C.c_float), ("pitch_limit", C.c_float), ("move_speed", C.c_float),
                ("move_speed_change_step", C.c_float), ("fps_limit", C.c_float), ("restrict_frame_count", C.c_uint32),
                ("target_frame_us", C.c_int64), ("sleep_margin_us", C.c_int64), ("relative_mouse", C.c_uint32),
                ("reserved", C.c_uint32)]


class InputState(C.Structure):
    """rt_input_state: KeyMouseInputArgs (SDL_OpenGLWindow.cuh:47-60) for one frame."""
    _fields_ = [("key_w", C.c_uint32), ("key_a", C.c_uint32), ("key_s", C.c_uint32), ("key_d", C.c_uint32),
                ("key_space", C.c_uint32), ("key_lshift", C.c_uint32), ("dx", C.c_int32), ("dy", C.c_int32),
                ("d_speed", C.c_int32), ("mouse_click", C.c_uint32), ("key_quit", C.c_uint32)]


class VtkInfo(C.Structure):
    _fields_ = [("point_count", C.c_uint64), ("particle_count", C.c_uint64),
                ("strip_vertex_count", C.c_uint64), ("triangle_count", C.c_uint64)]


class VtkParticle(C.Structure):
    _fields_ = [("id", C.c_uint64), ("velocity", Vec3), ("bounds", C.c_float * 6), ("centroid", Vec3),
                ("first_vertex", C.c_uint32), ("vertex_count", C.c_uint32)]


# Every symbol include/rt.h declares; tests check the library exports all of them.
EXPORTED_SYMBOLS = (
    "rt_abi_version", "rt_last_error", "rt_device_count", "rt_scene_create", "rt_scene_build",
    "rt_camera_set", "rt_scene_update", "rt_render", "rt_assemble_tiles", "rt_tiles_for_rank",
    "rt_trace_rays", "rt_synchronize", "rt_scene_destroy", "rt_scene_get_info",
    "rt_scene_export_blas", "rt_scene_export_tlas", "rt_demo_update", "rt_scene_set_option",
    "rt_scene_collect", "rt_scene_debug_read", "rt_scene_update_triangles", "rt_scene_update_instances",
    "rt_vtk_read", "rt_vtk_free", "rt_vtk_get_info", "rt_vtk_particles", "rt_vtk_vertices", "rt_vtk_convert",
    "rt_vtk_series_read", "rt_vtk_series_count", "rt_vtk_series_entry", "rt_vtk_series_free",
    "rt_comm_unique_id", "rt_scene_attach_comm", "rt_scene_detach_comm", "rt_slab_tiles", "rt_tile_pixels",
    "rt_comm_set_timeout", "rt_camera_control_init", "rt_camera_move", "rt_clock_ns", "rt_frame_pace",
    "rt_box_test",
)

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.path.join(PKG_DIR, "lib", "librtamd.so")


class RtError(RuntimeError):
    pass


def _declare(lib):
    P = C.POINTER
    lib.rt_abi_version.restype = C.c_uint32
    lib.rt_last_error.restype = C.c_char_p
    lib.rt_device_count.restype = C.c_int
    lib.rt_scene_create.argtypes = [P(SceneDesc), C.c_int, P(C.c_void_p)]
    lib.rt_scene_build.argtypes = [C.c_void_p, C.c_int, C.c_uint64]
    lib.rt_camera_set.argtypes = [C.c_void_p, P(CameraInput), C.c_uint32, C.c_uint32]
    lib.rt_scene_update.argtypes = [C.c_void_p, C.c_uint64]
    lib.rt_render.argtypes = [C.c_void_p, C.c_uint64, P(RenderOpts), C.c_void_p, C.c_void_p, P(Stats)]
    lib.rt_assemble_tiles.argtypes = [C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint32, C.c_uint32,
                                      C.c_uint32, C.c_void_p, C.c_void_p]
    lib.rt_tiles_for_rank.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32]
    lib.rt_tiles_for_rank.restype = C.c_uint32
    lib.rt_trace_rays.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_uint32, P(Hit)]
    lib.rt_box_test.argtypes = [C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t, C.c_uint32, C.c_void_p, C.c_void_p]
    lib.rt_box_test.restype = C.c_int
    lib.rt_synchronize.argtypes = [C.c_void_p]
    lib.rt_scene_destroy.argtypes = [C.c_void_p]
    lib.rt_scene_destroy.restype = None
    lib.rt_scene_get_info.argtypes = [C.c_void_p, P(SceneInfo)]
    lib.rt_scene_export_blas.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p, C.c_void_p,
                                         P(C.c_uint32), P(C.c_uint32)]
    lib.rt_scene_export_tlas.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                         P(C.c_uint32), P(C.c_uint32)]
    for name in ("rt_scene_create", "rt_scene_build", "rt_camera_set", "rt_scene_update", "rt_render",
                 "rt_assemble_tiles", "rt_trace_rays", "rt_synchronize", "rt_scene_get_info",
                 "rt_scene_export_blas", "rt_scene_export_tlas"):
        getattr(lib, name).restype = C.c_int
    lib.rt_scene_collect.argtypes = [C.c_void_p, P(Stats), P(C.c_float), C.c_uint32, P(C.c_uint32)]
    lib.rt_scene_collect.restype = C.c_int
    lib.rt_scene_set_option.argtypes = [C.c_void_p, C.c_char_p, C.c_int64]
    lib.rt_scene_set_option.restype = C.c_int
    lib.rt_scene_debug_read.argtypes = [C.c_void_p, C.c_char_p, C.c_void_p, C.c_size_t, P(C.c_size_t)]
    lib.rt_scene_debug_read.restype = C.c_int
    lib.rt_scene_update_triangles.argtypes = [C.c_void_p, C.c_size_t, C.c_size_t, C.c_void_p]
    lib.rt_scene_update_triangles.restype = C.c_int
    lib.rt_scene_update_instances.argtypes = [C.c_void_p, C.c_size_t, C.c_size_t, P(InstanceDesc)]
    lib.rt_scene_update_instances.restype = C.c_int
    lib.rt_vtk_read.argtypes = [C.c_char_p, P(C.c_void_p)]
    lib.rt_vtk_free.argtypes = [C.c_void_p]
    lib.rt_vtk_free.restype = None
    lib.rt_vtk_get_info.argtypes = [C.c_void_p, P(VtkInfo)]
    lib.rt_vtk_particles.argtypes = [C.c_void_p, P(VtkParticle)]
    lib.rt_vtk_vertices.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p]
    lib.rt_vtk_convert.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p, P(InstanceDesc)]
    lib.rt_vtk_series_read.argtypes = [C.c_char_p, P(C.c_void_p)]
    lib.rt_vtk_series_count.argtypes = [C.c_void_p]
    lib.rt_vtk_series_count.restype = C.c_size_t
    lib.rt_vtk_series_entry.argtypes = [C.c_void_p, C.c_size_t, P(C.c_char_p), P(C.c_float)]
    lib.rt_vtk_series_free.argtypes = [C.c_void_p]
    lib.rt_vtk_series_free.restype = None
    for name in ("rt_vtk_read", "rt_vtk_get_info", "rt_vtk_particles", "rt_vtk_vertices", "rt_vtk_convert",
                 "rt_vtk_series_read", "rt_vtk_series_entry"):
        getattr(lib, name).restype = C.c_int
    lib.rt_comm_unique_id.argtypes = [P(CommId)]
    lib.rt_scene_attach_comm.argtypes = [C.c_void_p, P(CommId), C.c_int, C.c_int, C.c_uint32, C.c_uint32]
    lib.rt_scene_detach_comm.argtypes = [C.c_void_p]
    lib.rt_slab_tiles.argtypes = [C.c_uint32] * 5
    lib.rt_slab_tiles.restype = C.c_uint32
    lib.rt_tile_pixels.argtypes = [C.c_uint32] * 6 + [C.c_uint64, C.c_uint64, C.c_void_p]
    for name in ("rt_comm_unique_id", "rt_scene_attach_comm", "rt_scene_detach_comm", "rt_tile_pixels"):
        getattr(lib, name).restype = C.c_int
    lib.rt_comm_set_timeout.argtypes = [C.c_void_p, C.c_uint32]
    lib.rt_comm_set_timeout.restype = C.c_int
    lib.rt_camera_control_init.argtypes = [P(CameraControl), C.c_float, C.c_float, C.c_float, C.c_uint32, C.c_float]
    lib.rt_camera_control_init.restype = C.c_int
    lib.rt_camera_move.argtypes = [P(CameraInput), P(CameraControl), P(InputState), P(C.c_uint32)]
    lib.rt_camera_move.restype = C.c_int
    lib.rt_clock_ns.restype = C.c_int64
    lib.rt_frame_pace.argtypes = [P(CameraControl), C.c_int64]
    lib.rt_frame_pace.restype = C.c_int64
    lib.rt_demo_update.argtypes = [C.c_void_p, P(Xform), C.c_size_t, C.c_uint64]
    lib.rt_demo_update.restype = None
    return lib


_LIB = None


def load_library(path: str | None = None):
    """Load librtamd.so.  Raises if it is missing: there is no CPU fallback."""
    global _LIB
    if _LIB is not None and path is None:
        return _LIB
    p = path or os.environ.get("RTAMD_LIB") or LIB_PATH   # RTAMD_LIB: diagnostic builds (make DIAG=1)
    if not os.path.exists(p):
        raise RtError(f"librtamd.so not built ({p}); run __graft_entry__.build()")
    lib = _declare(C.CDLL(p, mode=C.RTLD_GLOBAL))
    if lib.rt_abi_version() != RT_ABI_VERSION:
        raise RtError("ABI version mismatch between rt.h mirror and librtamd.so")
    if path is None:
        _LIB = lib
    return lib


def check(lib, status):
    if status != RT_OK:
        msg = lib.rt_last_error()
        raise RtError(f"{RT_STATUS_NAMES.get(status, status)}: {msg.decode() if msg else ''}")
    return status
