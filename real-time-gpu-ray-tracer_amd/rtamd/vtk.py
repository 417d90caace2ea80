"""Scene ingestion from legacy VTK particle files over the C ABI (rt_vtk_*).

Mirrors the reference's VTKReader (src/Global/VTKReader.cu) and Renderer::configureVTKFiles
(src/Global/Renderer.cu:394-443):

    VTKReader::readVTKFile            -> VtkFile(path)            (particles, strip vertices, normals)
    VTKReader::convertToRendererData  -> VtkFile.convert(base)    (TRIANGLE_DTYPE array, instance dicts)
    Renderer::configureVTKFiles       -> read_series(path)        [(path, time), ...]
    main() with LOAD_VTK              -> vtk_scene(series_or_file) (demo scene + the first file's particles)
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import abi


class VtkFile:
    def __init__(self, path: str):
        self.lib = abi.load_library()
        h = C.c_void_p()
        abi.check(self.lib, self.lib.rt_vtk_read(path.encode(), C.byref(h)))
        self.h = h
        self.path = path
        info = abi.VtkInfo()
        abi.check(self.lib, self.lib.rt_vtk_get_info(self.h, C.byref(info)))
        self.point_count = int(info.point_count)
        self.particle_count = int(info.particle_count)
        self.strip_vertex_count = int(info.strip_vertex_count)
        self.triangle_count = int(info.triangle_count)

    def close(self):
        if getattr(self, "h", None):
            self.lib.rt_vtk_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def particles(self) -> np.ndarray:
        out = (abi.VtkParticle * max(1, self.particle_count))()
        abi.check(self.lib, self.lib.rt_vtk_particles(self.h, out))
        dt = np.dtype([("id", np.uint64), ("velocity", np.float32, 3), ("bounds", np.float32, 6),
                       ("centroid", np.float32, 3), ("first_vertex", np.uint32), ("vertex_count", np.uint32)])
        assert dt.itemsize == C.sizeof(abi.VtkParticle)
        return np.frombuffer(out, dtype=dt, count=self.particle_count).copy()

    def vertices(self):
        """(positions, normals) of the concatenated strip vertex stream, float32 [strip_vertex_count, 3]."""
        pos = np.zeros((self.strip_vertex_count, 3), np.float32)
        nrm = np.zeros((self.strip_vertex_count, 3), np.float32)
        abi.check(self.lib, self.lib.rt_vtk_vertices(self.h, pos.ctypes.data, nrm.ctypes.data))
        return pos, nrm

    def convert(self, triangle_index_base: int = 0):
        """-> (triangles[TRIANGLE_DTYPE], instances[list of dict]) as VTKReader::convertToRendererData."""
        from .scenes import TRIANGLE_DTYPE
        tris = np.zeros(self.triangle_count, dtype=TRIANGLE_DTYPE)
        ins = (abi.InstanceDesc * max(1, self.particle_count))()
        abi.check(self.lib, self.lib.rt_vtk_convert(self.h, triangle_index_base, tris.ctypes.data, ins))
        instances = []
        for i in range(self.particle_count):
            d = ins[i]
            instances.append(dict(type=int(d.primitive_type), index=int(d.primitive_index), count=int(d.primitive_count),
                                  bounds=tuple(float(x) for x in d.local_bounds),
                                  centroid=(d.local_centroid.x, d.local_centroid.y, d.local_centroid.z),
                                  shift=(d.xform.shift.x, d.xform.shift.y, d.xform.shift.z),
                                  rotate=(d.xform.rotate_deg.x, d.xform.rotate_deg.y, d.xform.rotate_deg.z),
                                  scale=(d.xform.scale.x, d.xform.scale.y, d.xform.scale.z)))
        return tris, instances


def read_series(path: str):
    """[(vtk file path, time)] of a .vtk.series index (Renderer::configureVTKFiles)."""
    lib = abi.load_library()
    h = C.c_void_p()
    abi.check(lib, lib.rt_vtk_series_read(path.encode(), C.byref(h)))
    try:
        out = []
        for i in range(lib.rt_vtk_series_count(h)):
            p, t = C.c_char_p(), C.c_float()
            abi.check(lib, lib.rt_vtk_series_entry(h, i, C.byref(p), C.byref(t)))
            out.append((p.value.decode(), float(t.value)))
        return out
    finally:
        lib.rt_vtk_series_free(h)


def vtk_scene(path: str):
    """Demo scene + the particles of a VTK file (or of the first file of a .vtk.series), merged
    like main() with LOAD_VTK (src/Global/Main.cu:109-115, Renderer.cu:9-121): particle
    triangles prepended, demo triangle instance indices shifted, particle instances appended."""
    from .scenes import demo_scene
    if path.endswith(".series"):
        path = read_series(path)[0][0]
    tris, inst = VtkFile(path).convert(0)
    s = demo_scene()
    n = tris.shape[0]
    s.triangles = np.concatenate([tris, s.triangles])
    for d in s.instances:
        if d["type"] == abi.TRIANGLE:
            d["index"] += n
    s.instances = s.instances + inst
    return s


class VtkSeriesPlayer:
    """Plays a .vtk.series through a Renderer built with mode="lbvh" from vtk_scene(series): frame k
    of the series replaces the particle triangles (rt_scene_update_triangles, BLASes rebuilt on the
    GPU) and the particle instances' bounds / centroids (rt_scene_update_instances).  An extension:
    the reference loads only the first file (Renderer.cu:13, :82).  Every file must keep the first
    file's particle / triangle counts."""

    def __init__(self, renderer, series_path: str, first_instance: int = 5):
        self.r = renderer
        self.entries = read_series(series_path)
        self.first_instance = first_instance

    def __len__(self):
        return len(self.entries)

    def load(self, k: int):
        tris, inst = VtkFile(self.entries[k][0]).convert(0)
        self.r.update_triangles(0, tris)
        self.r.update_instances(self.first_instance, inst)
        return self.entries[k][1]
