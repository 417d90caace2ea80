"""The trace kernels' box decisions against BoundingBox::hit (src/AS/BoundingBox.cu:34-72), through rt_box_test.

The FAST kernels cull with reciprocal-direction planes (one FMA per plane) and widen the interval by a bound on its
distance from the reference's, so a FAST cull never rejects a box the reference keeps; the exact-decision kernels
(binary pairs, quads of the reference's trees and, with option "exact_decisions", of GPU-built trees) re-take every
decision inside that margin with the reference's division slab.  Checked here per mode of include/rt.h `rt_box_mode`:

  * RT_BOX_REFERENCE (the EXACT kernel): hit flag and entry t bit-identical to the golden AABB KATs (oracle);
  * RT_BOX_DECIDE / RT_BOX_QUAD_PAIR: the same hit flags as the KATs, for every ray (the decisions of the W = 0 / 2 / 3
    instances), entry t within the margin (bit-identical wherever the decision was re-taken);
  * RT_BOX_CULL / RT_BOX_QUAD_GREEDY (host SAH and, by default, GPU-built trees): a superset of the KAT hits — never a
    missed hit the reference keeps but for the documented parallel-axis-on-a-face case; extras only inside the margin.

Beyond the 4 096 golden rays (10 % with a zero direction component): crafted rays with a parallel axis whose origin
lies exactly on a face, on an edge or a corner of the box (the reference keeps q == min / max, BoundingBox.cu:47),
rays exactly grazing a face (entry == exit: the reference's cmin >= cmax rejects), tiny but non-parallel components
on both sides of the 1e-6 threshold, and tmax equal to the entry t, one ulp above and below it (the pop re-test
compares entry t with tmax, Range.cuh:33-43 / BoundingBox.cu:66).  Expected answers: the oracle's oracle_hit_aabb
(tests only use it as the checker).
"""
import os

import numpy as np
import pytest

from rtamd.renderer import box_test

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
EXACT_MODES = ("decide", "quad_pair")
CULL_MODES = ("cull", "quad_greedy")


def oracle_boxes(boxes, rays, tmax):
    from oracle.oracle import lib
    n = len(boxes)
    hit = np.zeros(n, bool)
    te = np.full(n, np.inf, np.float32)
    t = np.zeros(1, np.float32)
    for i in range(n):
        b = np.ascontiguousarray(boxes[i], np.float32)
        r = np.ascontiguousarray(rays[i], np.float32)
        rg = np.asarray([0.001, tmax[i]], np.float32)
        if lib().oracle_hit_aabb(b.ctypes.data, r.ctypes.data, rg.ctypes.data, t.ctypes.data):
            hit[i] = True
            te[i] = t[0]
    return hit, te


def crafted(seed=7):
    """Parallel axes with the origin on faces / edges / corners, grazing rays, near-threshold components."""
    g = np.random.default_rng(seed)
    boxes, rays = [], []
    for _ in range(600):
        lo = g.uniform(-2, 2, 3).astype(np.float32)
        hi = (lo + g.uniform(0.05, 1.5, 3)).astype(np.float32)
        b = np.array([lo[0], hi[0], lo[1], hi[1], lo[2], hi[2]], np.float32)
        kind = g.integers(0, 6)
        o = g.uniform(-4, 4, 3).astype(np.float32)
        c = (lo + hi) / 2
        d = (c + g.normal(size=3) * 0.3 - o).astype(np.float32)
        if kind <= 2:                                  # 1..3 parallel axes, origin on a face of each
            axes = g.choice(3, size=kind + 1, replace=False)
            for a in axes:
                o[a] = lo[a] if g.random() < 0.5 else hi[a]
                d[a] = [0.0, 5e-7, -5e-7, 1e-20][g.integers(0, 4)]
            if (np.abs(d) < 1e-6).all():
                d[g.integers(0, 3)] = 1.0
        elif kind == 3:                                # grazing: the ray runs along a face plane
            a = g.integers(0, 3)
            o[a] = lo[a] if g.random() < 0.5 else hi[a]
            d[a] = 0.0
            b2 = (a + 1) % 3
            o[b2] = lo[b2] - 1.0
            d[b2] = 1.0
        elif kind == 4:                                # components on both sides of the 1e-6 threshold
            a = g.integers(0, 3)
            d[a] = np.float32([9.99e-7, 1.0001e-6, -1e-6, 1e-6][g.integers(0, 4)])
            o[a] = g.uniform(lo[a], hi[a])
        else:                                          # through an edge or a corner exactly
            tgt = np.array([lo[0] if g.random() < 0.5 else hi[0], lo[1] if g.random() < 0.5 else hi[1],
                            lo[2] if g.random() < 0.5 else hi[2]], np.float32)
            d = (tgt - o).astype(np.float32)
        boxes.append(b)
        rays.append(np.concatenate([o, d]).astype(np.float32))
    return np.asarray(boxes, np.float32), np.asarray(rays, np.float32)


@pytest.fixture(scope="module")
def cases():
    g = np.load(os.path.join(GOLDEN, "prim_kats.npz"))
    kb, kr, ko = g["aabb_boxes"], g["aabb_rays"], g["aabb_out"]
    cb, cr = crafted()
    boxes = np.concatenate([kb, cb])
    rays = np.concatenate([kr, cr])
    inf = np.full(len(boxes), np.inf, np.float32)
    h0, t0 = oracle_boxes(boxes, rays, inf)
    assert np.array_equal(h0[:len(kb)], ko[:, 0] > 0) and np.array_equal(t0[:len(kb)][h0[:len(kb)]], ko[h0[:len(kb)], 1])
    # tmax at the entry t of each hit and one ulp either side: the pop re-test's boundary
    hb = np.flatnonzero(h0)
    t_at = t0[hb]
    tb = np.concatenate([boxes, boxes[hb], boxes[hb], boxes[hb]])
    tr = np.concatenate([rays, rays[hb], rays[hb], rays[hb]])
    tm = np.concatenate([inf, t_at, np.nextafter(t_at, np.float32(np.inf)), np.nextafter(t_at, np.float32(0))])
    hit, te = oracle_boxes(tb, tr, tm)
    return tb, tr, tm, hit, te, len(boxes)


def test_reference_mode_equals_the_kats(gpu_lib, cases):
    b, r, tm, hit, te, _ = cases
    h, t = box_test(b, r, tm, "reference")
    assert np.array_equal(h, hit), int((h != hit).sum())
    assert np.array_equal(t[hit], te[hit])


@pytest.mark.parametrize("mode", EXACT_MODES)
def test_exact_decision_modes_equal_the_kats(gpu_lib, cases, mode):
    """The W = 0 / 2 / 3 instances' decisions: every hit flag the reference's (no FAST cull decision survives)."""
    b, r, tm, hit, te, _ = cases
    h, t = box_test(b, r, tm, mode)
    bad = np.flatnonzero(h != hit)
    assert bad.size == 0, (mode, bad.size, [(b[i].tolist(), r[i].tolist(), float(tm[i]), bool(hit[i])) for i in bad[:3]])
    m = hit & np.isfinite(te)
    rel = np.abs(t[m] - te[m]) / np.maximum(np.abs(te[m]), 1e-3)
    assert rel.max() <= 1e-5, float(rel.max())


def on_parallel_face(b, r):
    """Rays with a parallel axis (|d| < 1e-6) whose origin lies exactly on a face of the box on that axis."""
    o, d = r[:, :3], r[:, 3:]
    lo, hi = b[:, 0::2], b[:, 1::2]
    return ((np.abs(d) < 1e-6) & ((o == lo) | (o == hi))).any(axis=1)


@pytest.mark.parametrize("mode", CULL_MODES)
def test_cull_modes_never_miss_a_reference_hit(gpu_lib, cases, mode):
    """The greedy-quad (host SAH) instances cull conservatively: a superset of the reference's hits, but for the one
    documented exception (trace_kernel.hip RT_SLAB_CONS / XD_PAR): a ray with a parallel axis whose origin lies exactly
    on a face of that axis's slab, which the reference keeps (BoundingBox.cu:47) and reciprocal planes cannot represent.
    The crafted cases hold ~400 such rays; every reference hit outside that case is kept."""
    b, r, tm, hit, te, n0 = cases                              # the first n0 cases: tmax = +inf
    h, _ = box_test(b, r, tm, mode)
    miss = hit & ~h
    exc = on_parallel_face(b, r)
    assert not (miss & ~exc).any(), int((miss & ~exc).sum())
    print(f"{mode}: {int(miss.sum())} reference hits culled, all with a parallel axis and the origin on its face "
          f"({int((exc & hit).sum())} such hits)")
    assert (h[:n0] & ~hit[:n0]).sum() <= 0.02 * n0, int((h[:n0] & ~hit[:n0]).sum())   # extras only inside the margin


def test_box_test_rejects_bad_arguments(gpu_lib):
    from rtamd import abi
    lib = abi.load_library()
    z = np.zeros(6, np.float32)
    hit = np.zeros(1, np.uint8)
    te = np.zeros(1, np.float32)
    assert lib.rt_box_test(0, z.ctypes.data, z.ctypes.data, z.ctypes.data, 1, 9, hit.ctypes.data, te.ctypes.data) != 0
    assert lib.rt_box_test(0, None, None, None, 1, 0, None, None) != 0
    assert lib.rt_box_test(0, None, None, None, 0, 0, None, None) == 0
