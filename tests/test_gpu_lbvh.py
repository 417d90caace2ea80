"""RT_BUILD_LBVH: BLASes and the per-frame TLAS built on the GPU (lbvh.hip), through the C ABI.

* every GPU-built BLAS equals the numpy restatement (tests/lbvh_ref.py) of the builder over the
  oracle's primitive boxes, bit for bit (node boxes, topology, leaf order);
* every GPU-built TLAS is a valid tree over all instances whose boxes are exact unions;
* images traverse different trees than the reference's, so they are held to the FAST tolerance
  against the oracle (compat trees), as RT_BUILD_SAH is;
* rebuilding every frame is deterministic (same bytes), and rt_scene_update_triangles followed by
  the GPU rebuild gives the same frame as a scene created with the moved triangles.
"""
import ctypes as C

import numpy as np
import pytest

from lbvh_ref import check_tree, lbvh_tree
from rtamd import Renderer, abi, scenes

pytestmark = pytest.mark.gpu

THREADS = 16


def frac_within(a, b, lsb=1):
    d = np.abs(a.astype(np.int32) - b.astype(np.int32)).max(axis=-1)
    return float((d <= lsb).mean()), int(d.max())


def prim_items(scene, ptype, first, count):
    """Reference primitive boxes (oracle) and centroids of primitives [first, first + count)."""
    from oracle.oracle import lib
    boxes = np.zeros((count, 6), np.float32)
    cents = np.zeros((count, 3), np.float32)
    f = np.float32
    for k in range(count):
        i = first + k
        if ptype == abi.TRIANGLE:
            t = scene.triangles[i]
            prim = abi.Triangle.from_buffer_copy(t.tobytes())
            v = t["vertex"].astype(np.float32)
            cents[k] = ((v[0] + v[1]) + v[2]) / f(3.0)
        elif ptype == abi.SPHERE:
            mt, mi, c, r = scene.spheres[i]
            prim = abi.Sphere(abi.Vec3.of(c), float(r), mt, mi)
            cents[k] = np.asarray(c, np.float32)
        else:
            mt, mi, q, u, v = scene.parallelograms[i]
            prim = abi.Parallelogram(abi.Vec3.of(q), abi.Vec3.of(u), abi.Vec3.of(v), mt, mi)
            q, u, v = (np.asarray(x, np.float32) for x in (q, u, v))
            cents[k] = (q + u * f(0.5)) + v * f(0.5)
        lib().oracle_prim_bounds(ptype, C.byref(prim), boxes[k].ctypes.data)
    return boxes, cents


def unique_blas(scene):
    """(type, first, count) per unique BLAS in instance order (RenderPin.cu:99-201 dedup)."""
    seen, out = set(), []
    for d in scene.instances:
        key = (d["type"], d["index"])
        if key not in seen:
            seen.add(key)
            out.append((d["type"], d["index"], d.get("count", 0) or 1))
    return out


def test_blas_trees_equal_restatement(gpu_lib):
    s = scenes.demo_with_particles(5)
    r = Renderer(s).set_option("group", 0).build_acceleration_structure(0, mode="lbvh").configure_camera(64, 64)
    blas = unique_blas(s)
    assert r.info()["blas_count"] == len(blas)
    for b, (ptype, first, count) in enumerate(blas):
        boxes, cents = prim_items(s, ptype, first, count)
        nb, ci, refs = r.export_blas(b)
        wb, wci, wrefs = lbvh_tree(boxes, cents, 4)
        assert np.array_equal(ci, wci), b
        assert np.array_equal(refs, wrefs + first), b
        assert np.array_equal(nb, wb), b
        check_tree(nb, ci, refs - first, boxes, 4)


def test_tlas_valid_every_frame(gpu_lib):
    s = scenes.demo_with_particles(12)
    r = Renderer(s).set_option("group", 0).build_acceleration_structure(0, mode="lbvh").configure_camera(64, 64)
    n = len(s.instances)
    for frame in (0, 5, 37):
        r.update(frame)
        nb, ci, refs = r.export_tlas()
        assert sorted(refs.tolist()) == list(range(n))
        # leaves <= 2 instances; interior boxes are exact unions of their children
        todo = [0]
        while todo:
            j = todo.pop()
            if ci[j, 0]:
                assert ci[j, 0] <= 2
                continue
            k = int(ci[j, 1])
            u = np.empty(6, np.float32)
            u[0::2] = nb[k:k + 2, 0::2].min(axis=0)
            u[1::2] = nb[k:k + 2, 1::2].max(axis=0)
            assert np.array_equal(nb[j], u), (frame, j)
            todo += [k, k + 1]
        assert r.info()["tlas_node_pairs"] == int((ci[:, 0] == 0).sum())


@pytest.mark.parametrize("depth,need", [(1, 0.999), (2, 0.999), (4, 0.995)])
def test_lbvh_images_within_tolerance(gpu_lib, depth, need):
    from oracle.oracle import OracleScene
    s = scenes.demo_with_particles(16)
    r = Renderer(s).build_acceleration_structure(0, mode="lbvh").configure_camera(320, 180, ray_trace_depth=depth)
    o = OracleScene(s, build_seed=0)
    o.camera(320, 180, ray_trace_depth=depth)
    for frame in (0, 37):
        o.update(frame)
        orgb, orgba, ocnt = o.render(threads=THREADS)
        for exact in (True, False):
            rgba, rgb, st = r.render(frame, exact=exact, want_rgb=True, count_work=True)
            f, mx = frac_within(rgba, orgba)
            assert f >= need, (frame, exact, f, mx)
            assert abs(st["rays"] - ocnt["rays"]) <= 0.001 * ocnt["rays"]


def test_trace_rays_hits_match_oracle(gpu_lib):
    """Per-ray closest hits through GPU-built trees: same surface as the oracle's compat trees on
    >= 99.9 % of rays (ties within 1e-6 may resolve to another primitive)."""
    from oracle.oracle import OracleScene
    s = scenes.demo_with_particles(20)
    r = Renderer(s).build_acceleration_structure(0, mode="lbvh").configure_camera(64, 64)
    o = OracleScene(s, build_seed=0)
    rng = np.random.default_rng(5)
    n = 20000
    org = np.stack([rng.uniform(-6, 6, n), rng.uniform(0.5, 8, n), rng.uniform(6, 12, n)], 1)
    tgt = np.stack([rng.uniform(-2, 2, n), rng.uniform(3.5, 5.5, n), rng.uniform(-1, 1, n)], 1)
    rays = np.concatenate([org, tgt - org], 1).astype(np.float32)
    g = r.trace_rays(rays, exact=True)
    h, _ = o.trace(rays)
    same = (g["instance"] == h["instance"]) & (g["pindex"] == h["pindex"])
    assert same.mean() >= 0.999, same.mean()
    hit = same & (h["instance"] != 0xFFFFFFFF)
    assert np.array_equal(g["t"][hit], h["t"][hit])


def test_per_frame_rebuild_is_deterministic(gpu_lib):
    s = scenes.demo_with_particles(10)
    a = Renderer(s).build_acceleration_structure(0, mode="lbvh").configure_camera(256, 144, ray_trace_depth=2)
    b = Renderer(s).build_acceleration_structure(0, mode="lbvh").configure_camera(256, 144, ray_trace_depth=2)
    b.set_option("rebuild", 1)
    for frame in range(4):
        x = a.render(frame, want_rgb=True)
        y = b.render(frame, want_rgb=True)
        assert np.array_equal(x[1], y[1]) and x[2]["rays"] == y[2]["rays"], frame
    # pipelined frames with a rebuild each frame
    b.collect()
    for frame in range(6):
        b.render(frame, sync=False, want_rgba=False, keep_counters=frame > 0)
    acc, kms = b.collect()
    assert len(kms) == 6 and acc["rays"] > 0


def test_update_triangles_rebuilds(gpu_lib):
    s = scenes.demo_with_particles(8)
    moved = s.triangles.copy()
    n_p = 8 * 1024
    moved["vertex"][:n_p] += np.asarray([0.05, 0.0, -0.03], np.float32)
    r = Renderer(s).build_acceleration_structure(0, mode="lbvh").configure_camera(256, 144, ray_trace_depth=2)
    before = r.render(0, want_rgb=True)[1]
    r.update_triangles(0, moved[:n_p])
    after = r.render(0, want_rgb=True)[1]
    assert not np.array_equal(before, after)
    s2 = scenes.demo_with_particles(8)
    s2.triangles = moved
    fresh = Renderer(s2).build_acceleration_structure(0, mode="lbvh").configure_camera(256, 144, ray_trace_depth=2)
    assert np.array_equal(after, fresh.render(0, want_rgb=True)[1])


@pytest.mark.parametrize("group,L,sets", [(1, 3, 3), (0, 3, 3), (1, 6, 5), (1, 8, 8)])
def test_update_triangles_pipelined_frames(gpu_lib, group, L, sets):
    """Deforming geometry without a device drain: each frame moves the particles' triangles and is launched on
    one of L overlapped lanes without waiting; every frame equals the same sequence rendered synchronously
    (the staged triangle copy is ordered behind the BLAS builds that read the array, never behind traces; with
    "blas_sets" spare sets in rotation a rebuild writes only a set no trace in flight still reads)."""
    import torch
    s = scenes.demo_with_particles(8)
    n_p = 8 * 1024
    W, H = 256, 144
    F = max(9, 2 * L + 3)

    def deform(f):
        t = s.triangles[:n_p].copy()
        t["vertex"] += np.asarray([0.02 * f, 0.01 * (f % 3), -0.015 * f], np.float32)
        return t

    ref_r = Renderer(s).set_option("group", group).build_acceleration_structure(0, mode="lbvh").configure_camera(
        W, H, ray_trace_depth=2)
    ref = []
    for f in range(F):
        ref_r.update_triangles(0, deform(f))
        ref.append(ref_r.render(f)[0])
    ref_r.cleanup()
    assert not np.array_equal(ref[0], ref[F - 1])
    r = Renderer(s).set_option("group", group).set_option("blas_sets", sets).build_acceleration_structure(
        0, mode="lbvh").configure_camera(W, H, ray_trace_depth=2)
    r.set_option("overlap", L)
    lanes = [torch.cuda.Stream() for _ in range(L)]
    bufs = [torch.zeros(W * H * 4, dtype=torch.uint8, device="cuda") for _ in range(F)]
    torch.cuda.synchronize()
    for f in range(F):
        r.update_triangles(0, deform(f))
        r.render(f, want_rgba=False, rgba8_device=bufs[f].data_ptr(), stream=lanes[f % L].cuda_stream, sync=False)
    r.synchronize()
    torch.cuda.synchronize()
    for f in range(F):
        assert np.array_equal(bufs[f].cpu().numpy().reshape(H, W, 4), ref[f]), f
    r.cleanup()


@pytest.mark.parametrize("double,sets,cold", [(1, 3, 0), (1, 2, 0), (1, 3, 1), (1, 2, 1), (0, 3, 0), (0, 3, 1)])
def test_update_triangles_once_then_pipelined_frames(gpu_lib, double, sets, cold):
    """One rt_scene_update_triangles, then frames on three overlapped lanes without waiting: only the first frame
    enqueues the BLAS rebuild (on the scene stream); the frames after it on the other lanes build nothing and must
    still wait for it before their instance records, TLAS and trace read the new BLAS set.  Every
    frame equals the synchronous render of the same frame by a default scene (one set in place or 2 / 3 sets in
    rotation, "blas_double" / "blas_sets"; with or without TriCold records, "cold_records" — same pixels)."""
    import torch
    P = 200                                            # ~205 k triangles: a rebuild long enough to race with
    s = scenes.demo_with_particles(P)
    n_p = P * 1024
    W, H, F, L = 256, 144, 9, 3
    moved = s.triangles[:n_p].copy()
    moved["vertex"] += np.asarray([0.04, -0.02, 0.03], np.float32)
    ref_r = Renderer(s).build_acceleration_structure(0, mode="lbvh")
    ref_r.configure_camera(W, H, ray_trace_depth=2)
    ref_r.update_triangles(0, moved)
    ref = [ref_r.render(f)[0] for f in range(F)]
    ref_r.cleanup()
    r = Renderer(s).set_option("blas_double", double).set_option("blas_sets", sets).set_option("cold_records", cold)
    r.build_acceleration_structure(0, mode="lbvh")
    r.configure_camera(W, H, ray_trace_depth=2)
    r.set_option("overlap", L)
    lanes = [torch.cuda.Stream() for _ in range(L)]
    bufs = [torch.zeros(W * H * 4, dtype=torch.uint8, device="cuda") for _ in range(F)]
    torch.cuda.synchronize()
    for f in range(3):                                 # frames on the old triangles first: the lanes are warm
        r.render(f, want_rgba=False, rgba8_device=bufs[f].data_ptr(), stream=lanes[f % L].cuda_stream, sync=False)
    r.synchronize()
    torch.cuda.synchronize()
    r.update_triangles(0, moved)
    for f in range(F):
        r.render(f, want_rgba=False, rgba8_device=bufs[f].data_ptr(), stream=lanes[f % L].cuda_stream, sync=False)
    r.synchronize()
    torch.cuda.synchronize()
    for f in range(F):
        assert np.array_equal(bufs[f].cpu().numpy().reshape(H, W, 4), ref[f]), f
    r.cleanup()


def test_trace_after_triangle_update_needs_a_frame_update(gpu_lib):
    """After rt_scene_update_triangles the BLASes are rebuilt by the next frame update; a trace that skips it
    (RT_RENDER_SKIP_UPDATE, rt_trace_rays) would mix the old trees with the new triangles a hit reads
    (raw_tris), so it is refused with RT_ERR_STATE until a frame has run its update (include/rt.h)."""
    s = scenes.demo_with_particles(4)
    r = Renderer(s).build_acceleration_structure(0, mode="lbvh").configure_camera(64, 48, ray_trace_depth=2)
    a = r.render(0)[0]
    assert np.array_equal(r.render(0, skip_update=True)[0], a)
    moved = s.triangles[:1024].copy()
    moved["vertex"] += np.asarray([0.01, 0.0, 0.0], np.float32)
    r.update_triangles(0, moved)
    with pytest.raises(abi.RtError, match="RT_ERR_STATE"):
        r.render(0, skip_update=True)
    with pytest.raises(abi.RtError, match="RT_ERR_STATE"):
        r.trace_rays(np.asarray([[0.0, 2.0, 10.0, 0.0, 0.0, -1.0]], np.float32))
    b = r.render(0)[0]                                 # the update rebuilds the BLASes
    assert np.array_equal(r.render(0, skip_update=True)[0], b)
    r.cleanup()


def test_update_triangles_needs_lbvh(gpu_lib):
    s = scenes.demo_with_particles(2)
    r = Renderer(s).build_acceleration_structure(0, mode="sah").configure_camera(32, 32)
    with pytest.raises(abi.RtError):
        r.update_triangles(0, s.triangles[:4])
    with pytest.raises(abi.RtError):
        r.set_option("rebuild", 1)


def test_large_forest_c5_shape(gpu_lib):
    """1,000 particle BLASes (1.02 M triangles, the C5 shape at 1/10 scale): every primitive is in
    exactly one leaf of its BLAS, and a frame matches the oracle within the FAST tolerance."""
    from oracle.oracle import OracleScene
    P = 1000
    s = scenes.demo_with_particles(P)
    r = Renderer(s).set_option("group", 0).build_acceleration_structure(0, mode="lbvh").configure_camera(
        192, 108, ray_trace_depth=2)
    info = r.info()
    assert info["blas_count"] == 5 - 1 + P
    assert info["blas_leaves"] == info["blas_node_pairs"] + info["blas_count"]
    for b in (4, 500, P + 3):                 # BLAS 4 + p = particle p (triangles p*1024 ...)
        _, _, refs = r.export_blas(b)
        assert sorted(refs.tolist()) == list(range((b - 4) * 1024, (b - 3) * 1024))
    o = OracleScene(s, build_seed=0)
    o.camera(192, 108, ray_trace_depth=2)
    _, orgba, _ = o.render(threads=THREADS)
    rgba, _, _ = r.render(0)
    f, mx = frac_within(rgba, orgba)
    assert f >= 0.999, (f, mx)


def test_large_single_blas_device_wide_path(gpu_lib):
    """A 65,536-triangle BLAS (> 2048 items) is finished by the device-wide bottom-up kernel
    (write-through hand-offs across XCDs): still bit-identical to the restatement."""
    from oracle.oracle import OracleScene
    tris, inst = scenes.synth_particles(64, 1024, seed=3)
    s = scenes.demo_scene()
    s.animated = False
    s.triangles = np.concatenate([tris, s.triangles])
    for d in s.instances:
        if d["type"] == abi.TRIANGLE:
            d["index"] += tris.shape[0]
    s.instances.append(dict(type=abi.TRIANGLE, index=0, count=tris.shape[0], shift=(0.0, 4.0, 0.0),
                            rotate=(90.0, 0.0, 0.0), scale=(3.0, 3.0, 3.0)))
    r = Renderer(s, update=False).build_acceleration_structure(0, mode="lbvh").configure_camera(200, 120, ray_trace_depth=2)
    b = len(unique_blas(s)) - 1
    boxes, cents = prim_items(s, abi.TRIANGLE, 0, tris.shape[0])
    nb, ci, refs = r.export_blas(b)
    wb, wci, wrefs = lbvh_tree(boxes, cents, 4)
    assert np.array_equal(ci, wci) and np.array_equal(refs, wrefs) and np.array_equal(nb, wb)
    o = OracleScene(s, build_seed=0)
    o.camera(200, 120, ray_trace_depth=2)
    _, orgba, _ = o.render(threads=THREADS)
    rgba, _, _ = r.render(0, exact=True)
    f, mx = frac_within(rgba, orgba)
    assert f >= 0.999, (f, mx)


def test_adjacent_large_blases_share_chunks(gpu_lib):
    """Two BLASes of 3,000 and 5,000 triangles (both > 2048 items, so both take the chunked bottom-up: 1024-item
    chunks through LDS, then the chunk-crossing nodes device-wide), adjacent in item order so that one chunk holds
    items of both; rebuilt twice: every node of both trees equals the restatement bit for bit."""
    tris, _ = scenes.synth_particles(8, 1024, seed=5)
    s = scenes.demo_scene()
    s.animated = False
    s.triangles = np.concatenate([tris, s.triangles])
    for d in s.instances:
        if d["type"] == abi.TRIANGLE:
            d["index"] += tris.shape[0]
    s.instances.append(dict(type=abi.TRIANGLE, index=0, count=3000, shift=(0.0, 4.0, 0.0),
                            rotate=(90.0, 0.0, 0.0), scale=(3.0, 3.0, 3.0)))
    s.instances.append(dict(type=abi.TRIANGLE, index=3000, count=5000, shift=(2.0, 1.0, 0.0),
                            rotate=(0.0, 30.0, 0.0), scale=(2.0, 2.0, 2.0)))
    r = Renderer(s, update=False).build_acceleration_structure(0, mode="lbvh").configure_camera(160, 90)
    r.set_option("rebuild", 1)
    r.render(0)
    blases = unique_blas(s)
    for first, count in ((0, 3000), (3000, 5000)):
        b = next(k for k, (t, f, c) in enumerate(blases) if t == abi.TRIANGLE and f == first and c == count)
        boxes, cents = prim_items(s, abi.TRIANGLE, first, count)
        nb, ci, refs = r.export_blas(b)
        wb, wci, wrefs = lbvh_tree(boxes, cents, 4)
        assert np.array_equal(ci, wci), (first, count)
        assert np.array_equal(refs, wrefs + first) or np.array_equal(refs, wrefs), (first, count)
        assert np.array_equal(nb, wb), (first, count)


def test_rebuild_sah_then_lbvh_equals_fresh_lbvh(gpu_lib):
    """A scene built with SAH (instance records staged in TLAS slot order) and then rebuilt with LBVH
    must trace instance-ordered records again: frames and per-ray hits equal a fresh LBVH scene
    (the LBVH frame path left the slot-order flag of its frame block set)."""
    s = scenes.demo_with_particles(10)
    rays = np.concatenate([np.tile([[0.0, 2.0, 10.0]], (4000, 1)),
                           np.random.default_rng(5).normal(size=(4000, 3)) * [1, 0.5, 1] + [0, 0, -1]], 1)
    rays[:, 3:] /= np.linalg.norm(rays[:, 3:], axis=1, keepdims=True)
    fresh = Renderer(s).build_acceleration_structure(0, mode="lbvh").configure_camera(200, 120, ray_trace_depth=2)
    want = [fresh.render(f)[0] for f in range(5)]
    want_hits = fresh.trace_rays(rays)
    fresh.cleanup()
    r = Renderer(s).build_acceleration_structure(0, mode="sah").configure_camera(200, 120, ray_trace_depth=2)
    for f in range(5):                       # every frame block gets staged in slot order
        r.render(f)
    r.build_acceleration_structure(0, mode="lbvh")
    for f in range(5):
        assert np.array_equal(r.render(f)[0], want[f]), f
    got = r.trace_rays(rays)
    for k in ("t", "instance", "pindex", "ptype", "point", "normal"):
        assert np.array_equal(got[k], want_hits[k]), k


PAIR_DT = np.dtype([("c0", np.float32, 6), ("c1", np.float32, 6), ("ref0", np.uint32), ("ref1", np.uint32),
                    ("pad", np.uint32, 2)])
QUAD_DT = np.dtype([("lo_x", np.float32, 4), ("hi_x", np.float32, 4), ("lo_y", np.float32, 4), ("hi_y", np.float32, 4),
                    ("lo_z", np.float32, 4), ("hi_z", np.float32, 4), ("ref", np.uint32, 4), ("pad", np.uint32, 4)])
ROOT_DT = np.dtype([("box", np.float32, 6), ("ref", np.uint32), ("height", np.uint32)])
REF_LEAF, REF_INDEX = 1 << 31, (1 << 30) - 1


def _expected_quads(pairs, root_ref):
    """csrc/bvh_build.hpp flatten_tree_wide restated on the GPU's own node pairs: quad q rooted at pair q holds q's
    two binary levels as two halves — slots 0, 1 = the left child's children, 2, 3 = the right child's; a leaf child
    takes its half's first slot and the second is empty (REF_EMPTY) with a copy of its box."""
    out, todo = {}, ([root_ref & REF_INDEX] if not root_ref & REF_LEAF else [])
    while todo:
        q = todo.pop()
        p = pairs[q]
        box, ref = [], []
        for c, r in ((p["c0"], int(p["ref0"])), (p["c1"], int(p["ref1"]))):
            if r & REF_LEAF:
                box += [c.copy(), c.copy()]
                ref += [r, 0xFFFFFFFF]
            else:
                g = pairs[r & REF_INDEX]
                box += [g["c0"].copy(), g["c1"].copy()]
                ref += [int(g["ref0"]), int(g["ref1"])]
        out[q] = (box, ref)
        todo += [r & REF_INDEX for r in ref if r != 0xFFFFFFFF and not r & REF_LEAF]
    return out


@pytest.mark.parametrize("mode", ["particles", "large", "group80"])
def test_gpu_quad_collapse_equals_restatement(gpu_lib, mode):
    """RT_BUILD_LBVH trees get the 4-wide form on the GPU (collapse_wide_kernel, lbvh.hip): every quad equals
    the host collapse rule applied to the GPU's binary tree (bit for bit, slot order included), and the quad
    traversal — which visits the binary tree's order — renders the binary traversal's frame within the FAST
    tolerance, with the same ray count."""
    if mode == "particles":
        s = scenes.demo_with_particles(12)
    elif mode == "group80":  # one 81,920-triangle group BLAS (> 65,536 items): collapsed one pair per thread
        s = scenes.demo_with_particles(80)
    else:   # one BLAS of 65k triangles: its frontier lives in global scratch, not LDS
        tris, inst = scenes.synth_particles(64, 1024, seed=3)
        s = scenes.demo_scene()
        s.triangles = np.concatenate([tris, s.triangles])
        for d in s.instances:
            if d["type"] == 2:
                d["index"] += tris.shape[0]
        s.instances.append(dict(type=2, index=0, count=tris.shape[0], shift=(0.0, 4.0, 0.0), rotate=(90.0, 0.0, 0.0),
                                scale=(3.0, 3.0, 3.0)))
    r = Renderer(s).build_acceleration_structure(0, mode="lbvh").configure_camera(240, 136, ray_trace_depth=2)
    pairs = r.debug_read("blas_pairs").view(PAIR_DT)
    quads = r.debug_read("blas_quads").view(QUAD_DT)
    roots = r.debug_read("blas_roots").view(ROOT_DT)
    n_quads = 0
    for b in range(len(roots)):
        for q, (box, ref) in _expected_quads(pairs, int(roots[b]["ref"])).items():
            g = quads[q]
            assert list(g["ref"]) == ref, (b, q)
            for k in range(4):
                got = [g["lo_x"][k], g["hi_x"][k], g["lo_y"][k], g["hi_y"][k], g["lo_z"][k], g["hi_z"][k]]
                assert np.array_equal(np.asarray(got, np.float32), box[k]), (b, q, k)
            n_quads += 1
    assert n_quads > 0
    out = {}
    for wide in (0, 1):
        r.set_option("wide", wide)
        out[wide] = r.render(3, count_work=True)
    f, mx = frac_within(out[0][0], out[1][0])
    assert f >= 0.999, (f, mx)
    assert abs(out[0][2]["rays"] - out[1][2]["rays"]) <= 0.001 * out[0][2]["rays"]
    assert out[1][2]["aabb_tests"] != out[0][2]["aabb_tests"]          # the quad form really ran


@pytest.mark.parametrize("group", [0, 1])
def test_small_tlas_equals_multi_kernel_tlas(gpu_lib, group):
    """Option "tlas_small": one workgroup builds the GPU TLAS (deltas, records, Morton, sort, Karras, boxes, pairs,
    quads, slots) when at most 512 records are in it.  Without instance groups every record is in the TLAS and the
    tree is the multi-kernel builder's: identical exports and byte-identical frames over animated frames.  With
    groups the inactive member records are left out of the TLAS altogether: the tree holds the live records only
    and frames stay within the FAST tolerance of the multi-kernel path (which sorts them into a dead subtree)."""
    s = scenes.demo_with_particles(12)
    a = Renderer(s).set_option("group", group).build_acceleration_structure(0, mode="lbvh").configure_camera(
        256, 144, ray_trace_depth=2)
    b = Renderer(s).set_option("group", group).build_acceleration_structure(0, mode="lbvh").configure_camera(
        256, 144, ray_trace_depth=2)
    b.set_option("tlas_small", 0)
    n = len(s.instances)
    for frame in (0, 3, 37):
        fa, fb = a.render(frame)[0], b.render(frame)[0]
        ta, tb = a.export_tlas(), b.export_tlas()
        if group == 0:
            assert np.array_equal(fa, fb), frame
            for x, y in zip(ta, tb):
                assert np.array_equal(x, y), frame
            assert sorted(ta[2].tolist()) == list(range(n))
        else:
            f, mx = frac_within(fa, fb)
            assert f >= 0.9995, (frame, f, mx)
            live = sorted(ta[2].tolist())
            assert live == list(range(n - 12)) + [n], live         # the demo instances and the group record
    a.cleanup()
    b.cleanup()


@pytest.mark.parametrize("rebuild", [0, 1])
def test_cold_records_auto_same_frames(gpu_lib, rebuild):
    """Option "cold_records" auto (-1): cold triangle records when the GPU-built BLASes are built once, none with a
    per-frame rebuild ("rebuild" set before the build).  Every policy renders the same bytes, FAST and EXACT, and the
    auto build holds TriCold records exactly when it should (device_bytes)."""
    s = scenes.demo_with_particles(6)
    frames = {}
    dev = {}
    for cold in (-1, 0, 1):
        r = Renderer(s).set_option("cold_records", cold).set_option("rebuild", rebuild)
        r.build_acceleration_structure(0, mode="lbvh").configure_camera(96, 64, ray_trace_depth=2)
        frames[cold] = [r.render(f, exact=e)[0] for f in (0, 37) for e in (False, True)]
        dev[cold] = r.info()["device_bytes"]
        r.cleanup()
    for cold in (0, 1):
        for a, b in zip(frames[-1], frames[cold]):
            assert np.array_equal(a, b), cold
    assert dev[-1] == (dev[0] if rebuild else dev[1]), dev
    # device_bytes counts the builder's workspace since round 6: without cold records the prep kernel
    # stages the TriHot records in item order (48 B per triangle), as many bytes as one set of TriCold records, so
    # only the per-frame rebuild's spare BLAS sets (each with TriCold records when cold) make cold records cost more
    assert dev[0] != dev[1], dev
    if rebuild:
        assert dev[1] > dev[0], dev


def test_rebuild_stage_timing(gpu_lib):
    """Option "timeline" times the GPU BLAS rebuild's stages (bench.py's "rebuild" roofline block): after a timed
    rebuild rt_scene_debug_read("rebuild_stages") gives the forest's items, interior nodes, node pairs, items in
    large trees (> 2048 items) and large trees, and a positive duration per stage; after an untimed rebuild it
    refuses rather than return the older figures."""
    s = scenes.demo_with_particles(6)
    r = Renderer(s).set_option("rebuild", 1).build_acceleration_structure(0, mode="lbvh").configure_camera(
        64, 48, ray_trace_depth=2)
    r.render(0)
    r.set_option("timeline", 1)
    r.update(1)
    v = r.debug_read("rebuild_stages").view(np.float64)
    n_items = sum(1024 for _ in range(6))
    assert len(v) == 5 + 9 and v[0] >= n_items and 0.9 * v[0] < v[1] <= v[0] and 0 < v[2] <= v[1]
    assert 0 <= v[3] <= v[0] and v[4] <= max(1.0, v[3] / 2049)
    assert (v[5:] > 0).all(), v
    r.set_option("timeline", 0)
    r.update(2)
    with pytest.raises(abi.RtError, match="RT_ERR_STATE"):
        r.debug_read("rebuild_stages")
    r.cleanup()
