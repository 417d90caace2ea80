"""Option "group" (RT_BUILD_SAH, host-built TLAS): triangle instances with bit-identical transforms share
one SAH BLAS over all their triangles and enter the TLAS as one item.  The reference keeps
one instance per VTK particle, all with the same fixed transform (VTKReader.cu:204-215, Renderer.cu:112-114);
a hit inside the group is the same closest hit in the same instance space, so:

  * images stay within the FAST tolerance of the oracle (which traverses the reference's per-instance
    trees), EXACT images too (same transform, closest hit equal up to 1e-6 ties);
  * per-ray hits report the member instance and primitive the oracle reports (>= 99.9 % of rays);
  * a frame in which a member's transform differs from the group's renders with per-instance items again:
    byte-identical to the same scene built without groups.
"""
import numpy as np
import pytest

from rtamd import Renderer, scenes

pytestmark = pytest.mark.gpu

THREADS = 16


def frac_within(a, b, lsb=1):
    d = np.abs(a.astype(np.int32) - b.astype(np.int32)).max(axis=-1)
    return float((d <= lsb).mean()), int(d.max())


def _rays(n, seed):
    """Rays aimed at the particle cluster (world y ~ 4, x / z in [-1.5, 1.5]) and around it."""
    g = np.random.default_rng(seed)
    o = np.stack([g.uniform(-3, 3, n), g.uniform(0.5, 8, n), g.uniform(4, 12, n)], 1)
    tgt = np.stack([g.uniform(-1.6, 1.6, n), g.uniform(2.4, 5.6, n), g.uniform(-1.6, 1.6, n)], 1)
    d = tgt - o
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    return np.concatenate([o, d], 1).astype(np.float32)


def test_group_images_and_hits_match_oracle(gpu_lib):
    from oracle.oracle import OracleScene
    s = scenes.demo_with_particles(24)
    W, H = 320, 180
    r = Renderer(s).build_acceleration_structure(0, mode="sah").configure_camera(W, H, ray_trace_depth=2)
    r0 = Renderer(s).set_option("group", 0).build_acceleration_structure(0, mode="sah").configure_camera(
        W, H, ray_trace_depth=2)
    assert r.info()["blas_count"] == r0.info()["blas_count"] == 4 + 24
    o = OracleScene(s, build_seed=0)
    o.camera(W, H, ray_trace_depth=2)
    for frame in (0, 7):
        o.update(frame)
        orgb, orgba, ocnt = o.render(threads=THREADS)
        for exact in (False, True):
            rgba, _, st = r.render(frame, exact=exact, count_work=True)
            f, mx = frac_within(rgba, orgba)
            assert f >= 0.999, (frame, exact, f, mx)
            assert abs(st["rays"] - ocnt["rays"]) <= 0.001 * ocnt["rays"]
    rays = _rays(20000, 5)
    oh, _ = o.trace(rays)
    for exact in (False, True):
        h = r.trace_rays(rays, exact=exact)
        same = (h["instance"] == oh["instance"]) & (h["pindex"] == oh["pindex"])
        assert same.mean() >= 0.999, (exact, same.mean())
        hit = same & (oh["instance"] != 0xFFFFFFFF)
        assert (oh["instance"][hit] >= 5).sum() > 1000            # the rays do reach the particles
        assert np.all(np.abs(h["t"][hit] - oh["t"][hit]) <= 1e-4 * oh["t"][hit])


def test_broken_group_equals_ungrouped_scene(gpu_lib):
    """A member whose transform changes takes the group out of the TLAS: that frame equals the frame of the
    scene built without groups byte for byte (same per-instance items, same trees)."""
    s = scenes.demo_with_particles(16)
    W, H = 256, 144
    rg = Renderer(s).build_acceleration_structure(0, mode="sah").configure_camera(W, H, ray_trace_depth=2)
    r0 = Renderer(s).set_option("group", 0).build_acceleration_structure(0, mode="sah").configure_camera(
        W, H, ray_trace_depth=2)
    a, b = rg.render(3)[0], r0.render(3)[0]
    f, _ = frac_within(a, b)
    assert f >= 0.999
    k = len(s.instances) - 3                      # a particle instance
    moved = dict(s.instances[k])
    moved["shift"] = (0.05, 4.0, 0.0)
    for rr in (rg, r0):
        rr.update_instances(k, [moved])
    for frame in (4, 5):
        assert np.array_equal(rg.render(frame)[0], r0.render(frame)[0]), frame
    for exact in (False, True):
        assert np.array_equal(rg.render(6, exact=exact)[0], r0.render(6, exact=exact)[0]), exact


# ---- option "group" with the GPU builder (RT_BUILD_LBVH): one LBVH segment over the members' triangles, in
# their leaf slots; members and the group are TLAS records, the inactive ones kept out of the GPU TLAS ----

def _lbvh(s, group=1, **cam):
    r = Renderer(s).set_option("group", group).build_acceleration_structure(0, mode="lbvh")
    return r.configure_camera(cam.pop("W", 320), cam.pop("H", 180), **cam)


def test_lbvh_group_tree_equals_restatement(gpu_lib):
    """The group's BLAS is the LBVH of the members' triangles taken as one contiguous range: equal bit for bit to
    the numpy restatement over the same primitives; a member's own BLAS is not built while the group holds."""
    from lbvh_ref import lbvh_tree
    from test_gpu_lbvh import prim_items
    from rtamd import abi
    P = 12
    s = scenes.demo_with_particles(P)
    r = _lbvh(s, W=64, H=64)
    nb_own = r.info()["blas_count"]
    assert nb_own == 4 + P
    boxes, cents = prim_items(s, abi.TRIANGLE, 0, P * 1024)
    nb, ci, refs = r.export_blas(nb_own)                  # the group's BLAS follows the own ones
    wb, wci, wrefs = lbvh_tree(boxes, cents, 4)
    assert np.array_equal(ci, wci) and np.array_equal(refs, wrefs) and np.array_equal(nb, wb)
    with pytest.raises(abi.RtError):
        r.export_blas(4)                                   # particle 0's own BLAS: not built
    n = len(s.instances)
    _, _, trefs = r.export_tlas()                         # the TLAS holds the demo instances and the group (record n)
    assert sorted(trefs.tolist()) == list(range(n - P)) + [n]
    r.set_option("tlas_small", 0)                         # the multi-kernel builder: every record is a leaf, the
    r.render(1)                                           # inactive ones in a subtree no ray enters
    _, _, trefs = r.export_tlas()
    assert sorted(trefs.tolist()) == list(range(n + 1))


def test_lbvh_group_images_and_hits_match_oracle(gpu_lib):
    from oracle.oracle import OracleScene
    s = scenes.demo_with_particles(24)
    r = _lbvh(s, ray_trace_depth=2)
    o = OracleScene(s, build_seed=0)
    o.camera(320, 180, ray_trace_depth=2)
    for frame in (0, 7):
        o.update(frame)
        _, orgba, ocnt = o.render(threads=THREADS)
        for exact in (False, True):
            rgba, _, st = r.render(frame, exact=exact, count_work=True)
            f, mx = frac_within(rgba, orgba)
            assert f >= 0.999, (frame, exact, f, mx)
            assert abs(st["rays"] - ocnt["rays"]) <= 0.001 * ocnt["rays"]
    rays = _rays(20000, 6)
    oh, _ = o.trace(rays)
    h = r.trace_rays(rays)
    same = (h["instance"] == oh["instance"]) & (h["pindex"] == oh["pindex"])
    assert same.mean() >= 0.999, same.mean()


@pytest.mark.parametrize("rebuild", [0, 1])
def test_lbvh_broken_group_switches_to_members(gpu_lib, rebuild):
    """A member moved by rt_scene_update_instances breaks the group for good: the builder switches to the
    members' own BLASes (exportable again) and the frame matches a scene built without groups within the
    FAST tolerance, with equal hits on >= 99.9 % of rays."""
    from rtamd import abi
    P = 16
    s = scenes.demo_with_particles(P)
    r = _lbvh(s, ray_trace_depth=2)
    r0 = _lbvh(s, group=0, ray_trace_depth=2)
    for x in (r, r0):
        x.set_option("rebuild", rebuild)
    first = len(s.instances) - P
    moved = dict(s.instances[first + 3])
    moved["shift"] = (0.3, 4.2, -0.1)
    for x in (r, r0):
        x.render(0)
        x.update_instances(first + 3, [moved])
    for frame in (1, 2):
        a, _, sa = r.render(frame, count_work=True)
        b, _, sb = r0.render(frame, count_work=True)
        f, mx = frac_within(a, b)
        assert f >= 0.9995, (frame, f, mx)
        assert abs(sa["instance_visits"] - sb["instance_visits"]) <= 0.01 * sb["instance_visits"]
    nb_own = r.info()["blas_count"]
    r.export_blas(first)                                   # a member's own BLAS is built now
    with pytest.raises(abi.RtError):
        r.export_blas(nb_own)                              # the group's is not
    rays = _rays(8000, 7)
    ha, hb = r.trace_rays(rays), r0.trace_rays(rays)
    assert ((ha["instance"] == hb["instance"]) & (ha["pindex"] == hb["pindex"])).mean() >= 0.999
