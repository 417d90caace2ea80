"""Scene descriptions for tests and benchmarks.

* ``demo_scene()`` restates the hard-coded scene of the reference's ``main``
  (src/Global/Main.cu:48-106): 2 spheres, 1 parallelogram, 1 triangle, 4 rough + 1 metal
  materials, 5 instances animated by ``updateInstance`` (Main.cu:6-42), camera 1200x800,
  FOV 90, 1 spp, depth 10.
* ``synth_particles(P, T, seed)`` is the synthetic stand-in for the VTK particle frames
  (SURVEY.md §8d): P closed UV-sphere meshes of T triangles, radius 0.05 +-20 %, placed in the
  VTK frame's local box, one instance each with the VTKReader transform (shift (0,4,0),
  rotate-x 90, scale 3; src/Global/VTKReader.cu:204-214) and material METAL 0.
  Particle triangles are inserted at the head of the triangle array and the demo triangle
  instance index is shifted, exactly as Renderer::commitGeometryData / configureInstances do
  with VTK data (src/Global/Renderer.cu:13-18, 101-108).
* ``CONFIGS`` restates BASELINE.json's five configs as concrete synthetic inputs.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, field

import numpy as np

from . import abi

# numpy twin of rt_triangle (include/rt.h) for building large meshes without Python loops
TRIANGLE_DTYPE = np.dtype([("vertex", np.float32, (3, 3)), ("normal", np.float32, (3, 3)),
                           ("material_type", np.uint32), ("material_index", np.uint32),
                           ("has_normals", np.uint32), ("reserved", np.uint32)])
assert TRIANGLE_DTYPE.itemsize == C.sizeof(abi.Triangle)

DEMO_CAMERA = dict(background=(0.7, 0.8, 0.9), center=(0.0, 2.0, 10.0), target=(0.0, 2.0, 0.0),
                   fov=90.0, up=(0.0, 1.0, 0.0), focus_disk_radius=0.0, sample_range=0.5,
                   sample_count=1, ray_trace_depth=10)                       # Main.cu:80-90
FRAME_SEED = 0x5EED


@dataclass
class Scene:
    """Host-side arrays of one scene (keeps the ctypes buffers alive)."""
    spheres: list
    parallelograms: list
    triangles: np.ndarray            # TRIANGLE_DTYPE
    roughs: list
    metals: list
    instances: list                  # list of dicts
    animated: bool = True            # apply the Main.cu updateInstance animation
    camera: dict = field(default_factory=lambda: dict(DEMO_CAMERA))
    _keep: list = field(default_factory=list, repr=False)

    @property
    def triangle_count(self):
        return int(self.triangles.shape[0])

    def desc(self, update_fn=None) -> abi.SceneDesc:
        """Build an rt_scene_desc; update_fn is a C function pointer (c_void_p) or None."""
        sph = (abi.Sphere * max(1, len(self.spheres)))()
        for i, (mt, mi, c, r) in enumerate(self.spheres):
            sph[i] = abi.Sphere(abi.Vec3.of(c), float(r), mt, mi)
        par = (abi.Parallelogram * max(1, len(self.parallelograms)))()
        for i, (mt, mi, q, u, v) in enumerate(self.parallelograms):
            par[i] = abi.Parallelogram(abi.Vec3.of(q), abi.Vec3.of(u), abi.Vec3.of(v), mt, mi)
        tri = np.ascontiguousarray(self.triangles, dtype=TRIANGLE_DTYPE)
        rou = (abi.Rough * max(1, len(self.roughs)))()
        for i, a in enumerate(self.roughs):
            rou[i] = abi.Rough(abi.Vec3.of(a))
        met = (abi.Metal * max(1, len(self.metals)))()
        for i, (a, f) in enumerate(self.metals):
            met[i] = abi.Metal(abi.Vec3.of(a), float(f))
        ins = instance_desc_array(self.instances)
        self._keep = [sph, par, tri, rou, met, ins]
        return abi.SceneDesc(
            C.cast(sph, C.POINTER(abi.Sphere)), len(self.spheres),
            C.cast(par, C.POINTER(abi.Parallelogram)), len(self.parallelograms),
            tri.ctypes.data_as(C.POINTER(abi.Triangle)), tri.shape[0],
            C.cast(rou, C.POINTER(abi.Rough)), len(self.roughs),
            C.cast(met, C.POINTER(abi.Metal)), len(self.metals),
            C.cast(ins, C.POINTER(abi.InstanceDesc)), len(self.instances),
            C.cast(update_fn, C.c_void_p) if update_fn is not None else None, None)

    def camera_input(self, **over) -> abi.CameraInput:
        c = dict(self.camera)
        c.update(over)
        return abi.CameraInput(abi.Vec3.of(c["background"]), abi.Vec3.of(c["center"]), abi.Vec3.of(c["target"]),
                               float(c["fov"]), abi.Vec3.of(c["up"]), float(c["focus_disk_radius"]),
                               float(c["sample_range"]), int(c["sample_count"]), int(c["ray_trace_depth"]))


def instance_desc_array(instances):
    """ctypes rt_instance_desc[] of instance dicts {type, index[, count, bounds, centroid, shift, rotate, scale]}."""
    ins = (abi.InstanceDesc * max(1, len(instances)))()
    for i, d in enumerate(instances):
        x = abi.Xform(abi.Vec3.of(d.get("shift", (0, 0, 0))), abi.Vec3.of(d.get("rotate", (0, 0, 0))),
                      abi.Vec3.of(d.get("scale", (1, 1, 1))))
        lb = d.get("bounds")
        ins[i] = abi.InstanceDesc(d["type"], d["index"], d.get("count", 0), 1 if lb is not None else 0,
                                  (C.c_float * 6)(*(lb if lb is not None else (0,) * 6)),
                                  abi.Vec3.of(d.get("centroid", (0, 0, 0))), x)
    return ins


def _demo_triangle():
    t = np.zeros(1, dtype=TRIANGLE_DTYPE)
    t["vertex"][0] = [[0.0, 0.0, 0.0], [1.0, 0.0, 1.0], [0.0, 1.0, 0.0]]              # Main.cu:56
    t["material_type"] = abi.ROUGH
    t["material_index"] = 2
    t["has_normals"] = 0
    return t


def demo_scene() -> Scene:
    """src/Global/Main.cu:48-99 without LOAD_VTK."""
    return Scene(
        spheres=[(abi.ROUGH, 3, (0.0, 0.0, 0.0), 1000.0), (abi.ROUGH, 0, (0.0, 0.0, 0.0), 2.0)],
        parallelograms=[(abi.ROUGH, 1, (0.0, 0.0, 0.0), (1.0, 0.0, 1.0), (0.0, 4.0, 0.0))],
        triangles=_demo_triangle(),
        roughs=[(.65, .05, .05), (.73, .73, .73), (.12, .45, .15), (.70, .60, .50)],
        metals=[((0.8, 0.85, 0.88), 0.0)],
        instances=[dict(type=abi.SPHERE, index=0), dict(type=abi.SPHERE, index=1),
                   dict(type=abi.PARALLELOGRAM, index=0), dict(type=abi.TRIANGLE, index=0),
                   dict(type=abi.SPHERE, index=1)],
    )


def uv_sphere_template(tris: int = 1024):
    """Unit UV sphere with `tris` triangles: 2*L*(S-1) with L slices, S stacks."""
    L = 32
    S = tris // (2 * L) + 1
    if 2 * L * (S - 1) != tris:
        raise ValueError("triangle count must be a multiple of 64")
    verts = [(0.0, 0.0, 1.0)]
    for i in range(1, S):
        th = np.pi * i / S
        for j in range(L):
            ph = 2.0 * np.pi * j / L
            verts.append((np.sin(th) * np.cos(ph), np.sin(th) * np.sin(ph), np.cos(th)))
    verts.append((0.0, 0.0, -1.0))
    verts = np.asarray(verts, dtype=np.float64)
    south = len(verts) - 1

    def ring(i, j):
        return 1 + (i - 1) * L + (j % L)

    faces = []
    for j in range(L):
        faces.append((0, ring(1, j), ring(1, j + 1)))
    for i in range(1, S - 1):
        for j in range(L):
            a, b, c, d = ring(i, j), ring(i, j + 1), ring(i + 1, j), ring(i + 1, j + 1)
            faces.append((a, c, b))
            faces.append((b, c, d))
    for j in range(L):
        faces.append((south, ring(S - 1, j + 1), ring(S - 1, j)))
    faces = np.asarray(faces, dtype=np.int64)
    assert len(faces) == tris
    return verts, faces


def _vertex_normals(verts, faces):
    """Area-weighted vertex normals (the build's stand-in for vtkPolyDataNormals,
    VTKReader.cu:60-70 — third-party boundary, parity unpinned there)."""
    p = verts[faces]
    fn = np.cross(p[:, 1] - p[:, 0], p[:, 2] - p[:, 0])
    vn = np.zeros_like(verts)
    for k in range(3):
        np.add.at(vn, faces[:, k], fn)
    vn /= np.linalg.norm(vn, axis=1, keepdims=True)
    return vn


def synth_particles(P: int, T: int = 1024, seed: int = 0x5EED):
    """P particles of T triangles each -> (triangles[P*T], instances[P])."""
    rng = np.random.Generator(np.random.PCG64(seed))
    verts, faces = uv_sphere_template(T)
    radius = 0.05 * (1.0 + 0.2 * (2.0 * rng.random(P) - 1.0))
    centers = np.stack([rng.uniform(-0.48, 0.46, P), rng.uniform(-0.48, 0.46, P),
                        rng.uniform(0.34, 0.47, P)], axis=1)
    tn = _vertex_normals(verts, faces)[faces].astype(np.float32)          # (T,3,3), radius-invariant
    tris = np.zeros(P * T, dtype=TRIANGLE_DTYPE)
    instances = []
    pos = (verts[None, :, :] * radius[:, None, None] + centers[:, None, :]).astype(np.float32)  # (P,V,3)
    tv = pos[:, faces]                                                    # (P,T,3,3)
    tris["vertex"] = tv.reshape(P * T, 3, 3)
    tris["normal"] = np.broadcast_to(tn, (P, T, 3, 3)).reshape(P * T, 3, 3)
    tris["material_type"] = abi.METAL
    tris["material_index"] = 0
    tris["has_normals"] = 1
    lo = pos.min(axis=1)
    hi = pos.max(axis=1)
    cen = pos.astype(np.float64).mean(axis=1).astype(np.float32)
    for p in range(P):
        instances.append(dict(type=abi.TRIANGLE, index=p * T, count=T,
                              bounds=(float(lo[p, 0]), float(hi[p, 0]), float(lo[p, 1]), float(hi[p, 1]),
                                      float(lo[p, 2]), float(hi[p, 2])),
                              centroid=tuple(float(c) for c in cen[p]),
                              shift=(0.0, 4.0, 0.0), rotate=(90.0, 0.0, 0.0), scale=(3.0, 3.0, 3.0)))
    return tris, instances


def demo_with_particles(P: int, T: int = 1024, seed: int = 0x5EED) -> Scene:
    """Demo scene + P synthetic particles, merged like the reference merges VTK data."""
    s = demo_scene()
    ptris, pinst = synth_particles(P, T, seed)
    n = ptris.shape[0]
    s.triangles = np.concatenate([ptris, s.triangles])                    # Renderer.cu:17
    for d in s.instances:
        if d["type"] == abi.TRIANGLE:
            d["index"] += n                                               # Renderer.cu:106-108
    s.instances = s.instances + pinst                                     # Renderer.cu:112-114
    return s


@dataclass(frozen=True)
class Config:
    name: str
    particles: int
    width: int
    height: int
    spp: int
    depth: int
    gpus: int
    description: str


# BASELINE.json "configs" restated.
CONFIGS = {
    "C1": Config("C1", 0, 256, 256, 1, 10, 0, "demo scene (Cornell stand-in), 256x256 1spp, host scalar"),
    "C2": Config("C2", 68, 1920, 1080, 1, 2, 1, "demo + 68x1024 tris (69,632; bunny stand-in), 1080p 1spp primary+shadow"),
    "C3": Config("C3", 254, 1920, 1080, 4, 4, 1, "demo + 254x1024 tris (260,096; Sponza stand-in), 1080p 4spp 3 bounces"),
    "C4": Config("C4", 254, 1920, 1080, 1, 2, 8, "C3 scene, 1080p 1spp, screen tiles over 8 GPUs + RCCL gather"),
    "C5": Config("C5", 9766, 3840, 2160, 8, 2, 8, "demo + 9766x1024 tris (~10M), 4K 8spp (4 traced)"),
}


def config_scene(cfg: Config) -> Scene:
    s = demo_scene() if cfg.particles == 0 else demo_with_particles(cfg.particles)
    s.camera["sample_count"] = cfg.spp
    s.camera["ray_trace_depth"] = cfg.depth
    return s


def demo_update_py(xforms, n, frame):
    """Python restatement of updateInstance (src/Global/Main.cu:6-42), float32 arithmetic.
    Used only to cross-check rt_demo_update; benchmarks use the native one."""
    f32 = np.float32
    angle = f32(frame) * f32(0.02)
    radius = f32(2.0)
    c, s_ = np.cos(angle, dtype=np.float32), np.sin(angle, dtype=np.float32)
    nc = (f32(0.0) + radius * c * f32(1.5), f32(2.0) + radius * s_ * c, f32(0.0) + radius * s_ * f32(1.5))
    nc2 = (-nc[0], nc[1], -nc[2])
    nc3 = (-nc[0], nc[1] + f32(5.0), nc[2])
    rot = f32(frame) * f32(0.4)
    table = [((0.0, -1000.0, 0.0), (0, 0, 0), (1, 1, 1)), (nc, (0, 0, 0), (1, 1, 1)),
             ((-5.0, 0.0, 0.0), (0, 0, 0), (1, 1, 1)), (nc2, (rot, rot, rot), (3, 3, 3)),
             (nc3, (0, 0, 0), (1, 1, 1))]
    for i, (sh, ro, sc) in enumerate(table[:min(n, 5)]):
        xforms[i] = abi.Xform(abi.Vec3.of(sh), abi.Vec3.of(ro), abi.Vec3.of(sc))
