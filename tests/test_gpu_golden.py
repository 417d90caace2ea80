"""HIP path vs the committed golden fixtures (no oracle needed at run time)."""
import os

import numpy as np
import pytest

from rtamd import Renderer, scenes

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
CROP = (72, 48, 96, 64)


@pytest.fixture(scope="module")
def vec():
    return np.load(os.path.join(GOLDEN, "scene_vectors.npz"))


def test_grid_hits_exact(gpu_lib, vec):
    r = Renderer(scenes.demo_with_particles(12)).build_acceleration_structure(5).configure_camera(64, 36)
    h = r.trace_rays(vec["grid_rays"], exact=True)
    for k in ("t", "instance", "ptype", "pindex", "point", "normal", "mtype", "midx"):
        assert np.array_equal(h[k], vec[f"grid_{k}"]), k


def test_bvh_dumps_identical(gpu_lib, vec):
    r = Renderer(scenes.demo_with_particles(12)).build_acceleration_structure(5).configure_camera(64, 36)
    nb = r.info()["blas_count"]
    b = r.export_blas(nb - 1)
    for x, k in zip(b, ("blas_boxes", "blas_ci", "blas_refs")):
        assert np.array_equal(x, vec[k]), k
    t = r.export_tlas()
    for x, k in zip(t, ("tlas_boxes", "tlas_ci", "tlas_refs")):
        assert np.array_equal(x, vec[k]), k


CASES = {
    "demo_d1": (scenes.demo_scene, dict(ray_trace_depth=1), 0),
    "demo_d2": (scenes.demo_scene, dict(ray_trace_depth=2), 0),
    "demo_d10": (scenes.demo_scene, dict(ray_trace_depth=10), 0),
    "demo_d10_f37": (scenes.demo_scene, dict(ray_trace_depth=10), 37),
    "demo_spp4_d4": (scenes.demo_scene, dict(ray_trace_depth=4, sample_count=4), 0),
    "particles_d2": (lambda: scenes.demo_with_particles(12), dict(ray_trace_depth=2), 0),
}


@pytest.mark.parametrize("name", sorted(CASES))
def test_image_crops(gpu_lib, vec, name):
    make, cam, frame = CASES[name]
    r = Renderer(make()).build_acceleration_structure(5).configure_camera(240, 160, **cam)
    x0, y0, w, h = CROP
    rgba, rgb, _ = r.render(frame, exact=True, want_rgb=True)
    assert np.array_equal(rgb[y0:y0 + h, x0:x0 + w], vec[f"img_{name}_rgb"])
    assert np.abs(rgba[y0:y0 + h, x0:x0 + w].astype(int) - vec[f"img_{name}_rgba"].astype(int)).max() <= 1
    fast, frgb, _ = r.render(frame, want_rgb=True)   # FAST on the reference's trees: bit-identical float RGB
    assert np.array_equal(frgb[y0:y0 + h, x0:x0 + w], vec[f"img_{name}_rgb"])
    d = np.abs(fast[y0:y0 + h, x0:x0 + w].astype(int) - vec[f"img_{name}_rgba"].astype(int)).max(axis=2)
    assert (d <= 1).all()


def _single_prim_scene(kind, prim):
    from rtamd import abi
    s = scenes.demo_scene()
    s.animated = False
    if kind == "sphere":
        s.spheres = [(abi.ROUGH, 0, prim.center.tuple(), prim.radius)]
        s.instances = [dict(type=abi.SPHERE, index=0)]
    elif kind == "quad":
        s.parallelograms = [(abi.ROUGH, 0, prim.q.tuple(), prim.u.tuple(), prim.v.tuple())]
        s.instances = [dict(type=abi.PARALLELOGRAM, index=0)]
    else:
        t = np.zeros(1, dtype=scenes.TRIANGLE_DTYPE)
        t["vertex"][0] = [prim.vertex[i].tuple() for i in range(3)]
        t["normal"][0] = [prim.normal[i].tuple() for i in range(3)]
        t["has_normals"] = prim.has_normals
        s.triangles = t
        s.instances = [dict(type=abi.TRIANGLE, index=0)]
    return s


@pytest.mark.parametrize("build", ["compat", "sah", "lbvh"])
@pytest.mark.parametrize("exact", [True, False])
@pytest.mark.parametrize("kind", ["sphere", "tri", "quad"])
def test_prim_kats_through_trace(gpu_lib, kind, exact, build):
    """The KAT rays traced through a one-primitive scene (identity instance), EXACT and FAST kernels, every builder:
    t bit-identical to the oracle's single-primitive hit function; the parallelogram's hits are additionally clipped
    by its q-centred box (Parallelogram.cu:48-50), so there the GPU hits must be exactly the KAT hits whose ray meets
    that box under the reference's slab — the FAST kernel's box decisions included (rt_trace_rays takes exact
    decisions: binary pairs, marginal decisions re-taken with the reference's slab)."""
    from rtamd import abi
    g = np.load(os.path.join(GOLDEN, "prim_kats.npz"))
    rays, out = g[f"{kind}_rays"], g[f"{kind}_out"]
    prims = {
        "sphere": abi.Sphere(abi.Vec3(0.3, -0.2, 0.1), 1.3, 0, 0),
        "quad": abi.Parallelogram(abi.Vec3(-1, -0.5, 0.2), abi.Vec3(2, 0.3, 0), abi.Vec3(0.2, 1.7, 0.4), 0, 0),
    }
    if kind == "tri":
        t = abi.Triangle()
        for i, v in enumerate(((-1, -1, 0.1), (1.2, -0.8, -0.2), (0.1, 1.1, 0.3))):
            t.vertex[i] = abi.Vec3(*v)
        for i, v in enumerate(((0, 0, 1), (0.3, 0, 0.95), (0, 0.3, 0.95))):
            t.normal[i] = abi.Vec3(*v)
        t.has_normals = 1
        prims["tri"] = t
    r = Renderer(_single_prim_scene(kind, prims[kind]), update=False).build_acceleration_structure(0, mode=build)
    h = r.trace_rays(rays, exact=exact)
    gpu_hit = h["instance"] != 0xFFFFFFFF
    kat_hit = out[:, 0] > 0
    if kind == "quad":
        # the BVH path tests the ray against the q-centred box first: a hit survives iff the ray
        # meets that box at all (oracle slab test, identical arithmetic in EXACT mode)
        import ctypes as C
        from oracle.oracle import lib
        box = np.zeros(6, np.float32)
        lib().oracle_prim_bounds(abi.PARALLELOGRAM, C.byref(prims["quad"]), box.ctypes.data)
        rg = np.asarray([0.001, np.inf], np.float32)
        te = np.zeros(1, np.float32)
        in_box = np.array([bool(lib().oracle_hit_aabb(box.ctypes.data, rays[i].ctypes.data, rg.ctypes.data,
                                                      te.ctypes.data)) for i in range(len(rays))])
        assert np.array_equal(gpu_hit, kat_hit & in_box)
        assert (kat_hit & ~in_box).sum() > 0                 # the bug is exercised
    else:
        assert np.array_equal(gpu_hit, kat_hit)
    m = gpu_hit
    assert np.array_equal(h["t"][m], out[m, 1])
    assert np.array_equal(h["point"][m], out[m, 2:5])
    assert np.abs(h["normal"][m] - out[m, 5:8]).max() <= 2e-7
    r.cleanup()
