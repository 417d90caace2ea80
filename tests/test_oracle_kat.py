"""Known-answer tests pinning the oracle (the CPU restatement of the reference).

The reference ships no tests or fixtures and cannot be built here, so these
analytic cases — derived by hand from the reference's formulas — are what pins the oracle.
Each case names the reference code it exercises.
"""
import math

import numpy as np
import pytest

from rtamd import abi, scenes

INF = float("inf")


def _ray(o, d):
    return np.asarray(list(o) + list(d), np.float32)


def _rng(lo, hi):
    return np.asarray([lo, hi], np.float32)


def hit(kind, prim, ray, rg=(0.001, INF)):
    from oracle.oracle import lib
    out = np.zeros(9, np.float32)
    fn = {"sphere": lib().oracle_hit_sphere, "quad": lib().oracle_hit_parallelogram,
          "tri": lib().oracle_hit_triangle}[kind]
    import ctypes as C
    r = fn(C.byref(prim), ray.ctypes.data, _rng(*rg).ctypes.data, out.ctypes.data)
    return bool(r), out


def sphere(c, r):
    return abi.Sphere(abi.Vec3.of(c), r, abi.ROUGH, 0)


def tri(a, b, c, normals=None):
    t = abi.Triangle()
    for i, v in enumerate((a, b, c)):
        t.vertex[i] = abi.Vec3.of(v)
    if normals is not None:
        for i, n in enumerate(normals):
            t.normal[i] = abi.Vec3.of(n)
        t.has_normals = 1
    return t


def quad(q, u, v):
    return abi.Parallelogram(abi.Vec3.of(q), abi.Vec3.of(u), abi.Vec3.of(v), abi.ROUGH, 0)


# ---- Sphere::hit (src/Geometry/Sphere.cu:4-49) -----------------------------------------
def test_sphere_front_hit(oracle_lib):
    ok, o = hit("sphere", sphere((0, 0, 0), 2.0), _ray((0, 0, 10), (0, 0, -1)))
    assert ok and o[0] == 8.0
    assert np.array_equal(o[1:4], [0, 0, 2]) and np.array_equal(o[4:7], [0, 0, 1])


def test_sphere_inside_takes_root2_and_flips_normal(oracle_lib):
    ok, o = hit("sphere", sphere((0, 0, 0), 2.0), _ray((0, 0, 0), (0, 0, 1)))
    assert ok and o[0] == 2.0
    assert np.array_equal(o[4:7], [0, 0, -1])          # outward normal flipped to face the ray


def test_sphere_miss_and_range(oracle_lib):
    assert not hit("sphere", sphere((0, 0, 0), 2.0), _ray((0, 3, 10), (0, 0, -1)))[0]
    # t = 8 outside [0.001, 7.5) and not within 1e-6 of either end -> root2 = 12 also out
    assert not hit("sphere", sphere((0, 0, 0), 2.0), _ray((0, 0, 10), (0, 0, -1)), (0.001, 7.5))[0]


def test_sphere_unnormalised_direction_scales_t(oracle_lib):
    ok, o = hit("sphere", sphere((0, 0, 0), 2.0), _ray((0, 0, 10), (0, 0, -2)))
    assert ok and o[0] == 4.0                          # t in units of |d| (Instance.cu:26-27 relies on it)


# ---- Range::inRange epsilon semantics (include/Util/Range.cuh:33-43) ----------------------
def test_range_right_end_epsilon_closed(oracle_lib):
    # tmax = 8 - 5e-7: t = 8 is within 1e-6 of tmax -> accepted ("later primitive wins ties")
    ok, o = hit("sphere", sphere((0, 0, 0), 2.0), _ray((0, 0, 10), (0, 0, -1)), (0.001, np.float32(8 - 5e-7)))
    assert ok and o[0] == 8.0
    ok, _ = hit("sphere", sphere((0, 0, 0), 2.0), _ray((0, 0, 10), (0, 0, -1)), (0.001, np.float32(8 - 4e-6)))
    assert not ok


# ---- Triangle::hit (src/Geometry/Triangle.cu:4-44) --------------------------------------
def test_triangle_barycentric_and_face_normal(oracle_lib):
    ok, o = hit("tri", tri((0, 0, 0), (1, 0, 0), (0, 1, 0)), _ray((0.25, 0.25, 5), (0, 0, -1)))
    assert ok and o[0] == 5.0 and o[7] == 0.25 and o[8] == 0.25
    assert np.array_equal(o[4:7], [0, 0, 1])


def test_triangle_back_side_flips_normal(oracle_lib):
    ok, o = hit("tri", tri((0, 0, 0), (1, 0, 0), (0, 1, 0)), _ray((0.25, 0.25, -5), (0, 0, 1)))
    assert ok and o[0] == 5.0 and np.array_equal(o[4:7], [0, 0, -1])


def test_triangle_edge_u_plus_v_equal_one_is_hit(oracle_lib):
    ok, o = hit("tri", tri((0, 0, 0), (1, 0, 0), (0, 1, 0)), _ray((0.5, 0.5, 5), (0, 0, -1)))
    assert ok and o[7] + o[8] == 1.0                   # `u + v > 1.0f` is strict


def test_triangle_outside_and_parallel(oracle_lib):
    assert not hit("tri", tri((0, 0, 0), (1, 0, 0), (0, 1, 0)), _ray((0.75, 0.75, 5), (0, 0, -1)))[0]
    assert not hit("tri", tri((0, 0, 0), (1, 0, 0), (0, 1, 0)), _ray((0.2, 0.2, 1), (1, 0, 0)))[0]


def test_triangle_interpolated_vertex_normals(oracle_lib):
    n0, n1, n2 = (0, 0, 1), (1, 0, 0), (0, 1, 0)
    ok, o = hit("tri", tri((0, 0, 0), (1, 0, 0), (0, 1, 0), (n0, n1, n2)), _ray((0.25, 0.25, 5), (0, 0, -1)))
    # n = unit(0.5*n0 + 0.25*n1 + 0.25*n2) = unit(0.25, 0.25, 0.5)
    exp = np.asarray([0.25, 0.25, 0.5]) / math.sqrt(0.375)
    assert ok and np.allclose(o[4:7], exp, atol=1e-6)


# ---- Parallelogram::hit (src/Geometry/Parallelogram.cu:4-46) ----------------------------
def test_parallelogram_alpha_beta(oracle_lib):
    ok, o = hit("quad", quad((0, 0, 0), (2, 0, 0), (0, 3, 0)), _ray((1, 1, 4), (0, 0, -1)))
    assert ok and o[0] == 4.0
    assert abs(o[7] - 0.5) < 1e-7 and abs(o[8] - 1.0 / 3.0) < 1e-7
    assert np.array_equal(o[4:7], [0, 0, 1])


def test_parallelogram_outside(oracle_lib):
    assert not hit("quad", quad((0, 0, 0), (2, 0, 0), (0, 3, 0)), _ray((3, 1, 4), (0, 0, -1)))[0]


# ---- AABBs (BoundingBox.cu:34-72, BoundingBox.cuh:24-47, Parallelogram.cu:48-50) ---------
def _aabb(box, ray, rg=(0.001, INF)):
    import ctypes as C
    from oracle.oracle import lib
    t = np.zeros(1, np.float32)
    r = lib().oracle_hit_aabb(np.asarray(box, np.float32).ctypes.data, ray.ctypes.data, _rng(*rg).ctypes.data,
                              t.ctypes.data)
    return bool(r), float(t[0])


def test_aabb_entry_t(oracle_lib):
    ok, t = _aabb([-1, 1, -1, 1, -1, 1], _ray((0, 0, 5), (0, 0, -1)))
    assert ok and t == 4.0


def test_aabb_parallel_axis_rules(oracle_lib):
    # d.x = 0 (< 1e-6): origin x outside the slab -> miss; inside -> axis skipped
    assert not _aabb([-1, 1, -1, 1, -1, 1], _ray((2, 0, 5), (0, 0, -1)))[0]
    assert _aabb([-1, 1, -1, 1, -1, 1], _ray((0.5, 0, 5), (0, 0, -1)))[0]


def test_aabb_tmax_culls(oracle_lib):
    assert not _aabb([-1, 1, -1, 1, -1, 1], _ray((0, 0, 5), (0, 0, -1)), (0.001, 4.0))[0]   # entry >= tmax
    assert _aabb([-1, 1, -1, 1, -1, 1], _ray((0, 0, 5), (0, 0, -1)), (0.001, 4.5))[0]


def _bounds(kind, prim):
    import ctypes as C
    from oracle.oracle import lib
    out = np.zeros(6, np.float32)
    lib().oracle_prim_bounds(kind, C.byref(prim), out.ctypes.data)
    return out


def test_parallelogram_box_is_centred_on_q_bug_compat(oracle_lib):
    # Main.cu:53 quad: q=(0,0,0), u=(1,0,1), v=(0,4,0) -> box q +- (u+v)/2 (not q + (u+v)/2 +- ..)
    b = _bounds(abi.PARALLELOGRAM, quad((0, 0, 0), (1, 0, 1), (0, 4, 0)))
    assert np.array_equal(b, np.asarray([-0.5, 0.5, -2, 2, -0.5, 0.5], np.float32))


def test_flat_triangle_box_gets_epsilon_volume(oracle_lib):
    b = _bounds(abi.TRIANGLE, tri((0, 0, 0), (1, 0, 0), (0, 1, 0)))
    assert b[4] == np.float32(-1e-6) and b[5] == np.float32(1e-6)


# ---- Matrix / Instance (src/Util/Matrix.cu, src/AS/Instance.cu:4-17) --------------------
def _mats(shift, rot, scale):
    from oracle.oracle import lib
    import ctypes as C
    out = np.zeros(48, np.float32)
    x = abi.Xform(abi.Vec3.of(shift), abi.Vec3.of(rot), abi.Vec3.of(scale))
    lib().oracle_instance_matrices(C.byref(x), out.ctypes.data)
    return out[:16].reshape(4, 4), out[16:32].reshape(4, 4), out[32:].reshape(4, 4)


def test_instance_matrices_shift_rotate_scale(oracle_lib):
    f, inv, nrm = _mats((0, 4, 0), (90, 0, 0), (3, 3, 3))         # VTKReader.cu:210-214 transform
    assert np.allclose(f @ np.asarray([0, 1, 0, 1], np.float32), [0, 4, 3, 1], atol=1e-5)  # y -> z
    assert np.allclose(f.astype(np.float64) @ inv.astype(np.float64), np.eye(4), atol=1e-6)
    assert np.array_equal(nrm, inv.T)


def test_instance_matrices_identity(oracle_lib):
    f, inv, nrm = _mats((0, 0, 0), (0, 0, 0), (1, 1, 1))
    assert np.array_equal(f, np.eye(4, dtype=np.float32)) and np.array_equal(inv, np.eye(4, dtype=np.float32))


# ---- RNG contract -------------------------------------------------------
def test_rng_contract_range_and_determinism(oracle_lib):
    from oracle.oracle import rng_stream
    a = rng_stream(1234 ^ 0x5EED, 1234, 4096)
    b = rng_stream(1234 ^ 0x5EED, 1234, 4096)
    assert np.array_equal(a, b)
    assert a.min() > 0.0 and a.max() <= 1.0
    assert abs(a.mean() - 0.5) < 0.02
    assert np.all(a * (1 << 24) == np.round(a * (1 << 24)))       # k / 2^24, k in 1..2^24
    c = rng_stream(1235 ^ 0x5EED, 1235, 4096)
    assert not np.array_equal(a, c)


def test_rng_contract_golden_prefix(oracle_lib):
    from oracle.oracle import rng_stream
    # splitmix64 finaliser contract: key = mix64(seed*G ^ (sub+1)*S), u = ((mix64(key + k*G) >> 40) + 1) / 2^24
    G, S, M = 0x9E3779B97F4A7C15, 0xD1B54A32D192ED03, (1 << 64) - 1

    def mix(z):
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M
        return z ^ (z >> 31)

    seed, sub = 77 ^ 0x5EED, 77
    key = mix(((seed * G) & M) ^ (((sub + 1) * S) & M))
    exp = [((mix((key + k * G) & M) >> 40) + 1) / float(1 << 24) for k in range(1, 9)]
    assert np.array_equal(rng_stream(seed, sub, 8), np.asarray(exp, np.float32))


# ---- Camera (src/Global/RenderPin.cu:73-95) -------------------------------------------------
def test_camera_demo_properties(oracle_lib):
    from oracle.oracle import OracleScene
    o = OracleScene(scenes.demo_scene())
    o.camera(1200, 800)
    c = o.camera_export()
    # FOV 90 horizontal, focus distance 10 -> viewport 20 x 13.333; W = -z, U = +x, V = +y
    po, dx, dy, center, U, V = c[0:3], c[3:6], c[6:9], c[9:12], c[12:15], c[15:18]
    assert np.allclose(U, [1, 0, 0]) and np.allclose(V, [0, 1, 0])
    assert np.allclose(dx, [20.0 / 1200, 0, 0], rtol=1e-6) and np.allclose(dy, [0, (20.0 * 800 / 1200) / 800, 0], rtol=1e-5)
    assert np.allclose(po, [-10 + 10.0 / 1200, 2 - 20.0 * 800 / 1200 / 2 + 0.5 * dy[1], 0], atol=1e-5)   # bottom-left
    assert np.array_equal(center, [0, 2, 10])
    o.camera(64, 64, sample_count=8)
    assert o.camera_export()[19] == 2.0                # floor(sqrt(8)) = 2 (RenderPin.cu:93)


# ---- Whole-path invariants -----------------------------------------------------------------
def test_primary_image_independent_of_tree_seed(oracle_lib):
    """Depth-1 images agree across random-axis trees except where two surfaces are within the
    1e-6 tie window (Range.cuh:33-43: the later-tested one wins), e.g. where the quad meets the
    ground; SURVEY.md fact 4 measured 0 such pixels on its scene, this scene has a handful."""
    from oracle.oracle import OracleScene
    imgs = []
    for seed in (1, 2, 99):
        o = OracleScene(scenes.demo_with_particles(8), build_seed=seed)
        o.camera(160, 90, ray_trace_depth=1)
        imgs.append(o.render(threads=4)[0])
    for other in imgs[1:]:
        diff = np.abs(imgs[0] - other).max(axis=2) > 0
        assert diff.mean() <= 1e-3


def test_bvh_matches_box_gated_brute_force(oracle_lib):
    """TLAS/BLAS traversal == loop over every instance/primitive gated by the primitive box
    (the NO_AS intent, Kernel.cu:10-62, plus the BVH's clipping), at depth 1."""
    from oracle.oracle import OracleScene
    o = OracleScene(scenes.demo_with_particles(4), build_seed=3)
    o.camera(120, 80, ray_trace_depth=1)
    a = o.render(threads=4)[0]
    b = o.render(threads=4, brute_force=2)[0]
    assert np.array_equal(a, b)


def test_unclipped_brute_force_shows_parallelogram_bug(oracle_lib):
    """Without the q-centred box (Parallelogram.cu:48-50) the quad is larger on screen."""
    from oracle.oracle import OracleScene
    o = OracleScene(scenes.demo_scene(), build_seed=3)
    o.camera(120, 80, ray_trace_depth=1)
    a = o.render(threads=4)[0]
    b = o.render(threads=4, brute_force=1)[0]
    assert (np.abs(a - b).max(axis=2) > 0).sum() > 0


def test_trace_counts_and_closest_hit(oracle_lib):
    from oracle.oracle import OracleScene
    o = OracleScene(scenes.demo_scene(), build_seed=0)
    hits, cnt = o.trace(np.asarray([[0, 2, 10, 0, -1, 0], [0, 2, 10, 0, 1, 0]], np.float32))
    assert cnt["rays"] == 2
    # ground: sphere r=1000 centred (0,-1000,0); below (0,*,10) its surface is at y = sqrt(1e6-100)-1000
    t_exp = 2.0 + 1000.0 - math.sqrt(1000.0 ** 2 - 100.0)
    assert hits["instance"][0] == 0 and abs(hits["t"][0] - t_exp) < 1e-3
    assert hits["instance"][1] == abi.MISS                                     # straight up: sky


# ---- C1 (BASELINE.json configs[0]): the demo scene at 256x256, BVH vs brute-force loops -------------------
@pytest.mark.parametrize("depth", [1, 2, 10])
def test_c1_bvh_equals_brute_force_256(oracle_lib, depth):
    """the demo scene (2 spheres, parallelogram, triangle; 5 instances) traced at 256x256 with the
    reference's TLAS/BLAS and with brute-force instance / primitive loops (the NO_AS intent of the dead
    Kernel.cu:10-62 path, gated by each primitive's own box as the BVH leaves are).  Primary rays are identical
    for every tree seed.  At depth >= 2 a bounce ray can hit two surfaces within the 1e-6 window, where the
    later-tested one wins (Range.cuh:33-43) and the loop order differs from the tree's: measured 0 pixels for
    tree seeds 1-5 and 1 (depth 2) / 2 (depth 10) of 65 536 for seed 0 (max 14 LSB) — inside SURVEY 8(c)'s
    0.01 % (depth 2) and 0.05 % (depth 10) outlier bars, which the test asserts."""
    from oracle.oracle import OracleScene
    bar = {1: 0, 2: 0.0001, 10: 0.0005}[depth]
    for seed in range(6):
        o = OracleScene(scenes.demo_scene(), build_seed=seed)
        o.camera(256, 256, ray_trace_depth=depth)
        a_rgb, a, ca = o.render(threads=4)
        b_rgb, b, cb = o.render(threads=4, brute_force=2)
        bad = (np.abs(a.astype(np.int32) - b.astype(np.int32)).max(axis=2) > 1).sum()
        assert bad <= bar * 256 * 256, (depth, seed, int(bad))
        if depth == 1:
            assert np.array_equal(a_rgb, b_rgb) and ca["rays"] == cb["rays"] == 256 * 256
        assert abs(ca["rays"] - cb["rays"]) <= 2
