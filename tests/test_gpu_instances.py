"""Per-frame instance update on the GPU (csrc/instances.hip).

GPU-built frames (RT_BUILD_LBVH) upload only the changed instances' (shift, cos / sin of the angles,
scale, local box); the GPU computes every instance's forward / inverse / inverse-transpose matrices and
transformed box and centroid each frame (Instance::updateTransformArguments, src/AS/Instance.cu:4-17;
Matrix.cu:101-130, 207-249; BoundingBox.cu:4-32).  The records must be bit-identical to the oracle's
host computation of the same frame, for every instance of the demo animation over 50 frames and of
the 9 771-instance C5 scene.
"""
import numpy as np
import pytest

from rtamd import Renderer, scenes

pytestmark = pytest.mark.gpu


def _gpu_records(r, n):
    return r.debug_read("instances").view(np.float32).reshape(n, 45)


def test_instance_records_bit_identical_50_frames(gpu_lib):
    from oracle.oracle import OracleScene
    s = scenes.demo_with_particles(12)
    n = len(s.instances)
    # option "group" off: with it the particles' own records are inactive (all-+inf boxes, kept out of the TLAS)
    r = Renderer(s).set_option("group", 0).build_acceleration_structure(0, mode="lbvh").configure_camera(64, 64)
    o = OracleScene(s, build_seed=0)
    for f in range(50):
        r.update(f)
        o.update(f)
        g, w = _gpu_records(r, n), o.instance_state()
        bad = np.flatnonzero((g.view(np.uint32) != w.view(np.uint32)).any(axis=1))
        assert bad.size == 0, (f, bad[:5], g[bad[0]] if bad.size else None, w[bad[0]] if bad.size else None)


def test_instance_records_c5_scene(gpu_lib):
    from oracle.oracle import OracleScene
    s = scenes.config_scene(scenes.CONFIGS["C5"])
    n = len(s.instances)
    assert n == 9771
    r = Renderer(s).set_option("group", 0).build_acceleration_structure(0, mode="lbvh").configure_camera(64, 64)
    o = OracleScene(s, build_seed=0)
    for f in (0, 1, 37):
        r.update(f)
        o.update(f)
        assert np.array_equal(_gpu_records(r, n).view(np.uint32), o.instance_state().view(np.uint32)), f


def test_instance_update_follows_update_instances(gpu_lib):
    """rt_scene_update_instances (new local bounds / transform, e.g. the next VTK frame) reaches the GPU
    records through the same delta path."""
    from oracle.oracle import OracleScene
    s = scenes.demo_with_particles(6)
    s.animated = False
    r = Renderer(s, update=False).build_acceleration_structure(0, mode="lbvh").configure_camera(64, 64)
    moved = [dict(d) for d in s.instances[5:8]]
    for d in moved:
        d["shift"] = (0.5, 3.0, -1.0)
        d["rotate"] = (10.0, 20.0, 30.0)
        lo = list(d["bounds"])
        d["bounds"] = (lo[0] - 0.01, lo[1], lo[2], lo[3] + 0.02, lo[4], lo[5])
    r.update_instances(5, moved)
    r.update(1)
    s2 = scenes.demo_with_particles(6)
    s2.animated = False
    s2.instances[5:8] = moved
    o = OracleScene(s2, build_seed=0)
    n = len(s.instances)
    assert np.array_equal(_gpu_records(r, n).view(np.uint32), o.instance_state().view(np.uint32))


def test_gpu_tlas_option_over_sah_blases(gpu_lib):
    """Option "gpu_tlas" (RT_BUILD_SAH BLASes, per-frame instance records + TLAS on the GPU): the records
    are bit-identical to the oracle's; the frames trace the same BLASes and instance records as the
    host-built TLAS, so only the TLAS shape differs and the pixels agree (closest hits tie only within
    the 1e-6 window)."""
    from oracle.oracle import OracleScene
    s = scenes.config_scene(scenes.CONFIGS["C2"])
    n = len(s.instances)
    W, H = 480, 270
    host = Renderer(s).build_acceleration_structure(0, mode="sah").configure_camera(W, H)
    dev = Renderer(s)
    dev.set_option("gpu_tlas", 1)
    dev.build_acceleration_structure(0, mode="sah").configure_camera(W, H)
    o = OracleScene(s, build_seed=0)
    for f in (0, 1, 7, 40):
        a, _, sa = host.render(f, count_work=True)
        b, _, sb = dev.render(f, count_work=True)
        o.update(f)
        assert np.array_equal(_gpu_records(dev, n).view(np.uint32), o.instance_state().view(np.uint32)), f
        # the same rays; a ray grazing a box edge may be culled by a different ancestor box (FAST slabs)
        assert abs(sa["rays"] - sb["rays"]) <= 2e-4 * sa["rays"], (f, sa["rays"], sb["rays"])
        assert abs(sa["hits"] - sb["hits"]) <= 2e-4 * sa["hits"], (f, sa["hits"], sb["hits"])
        same = float((a == b).all(axis=-1).mean())
        assert same >= 0.9995, (f, same)
    host.cleanup()
    dev.cleanup()
