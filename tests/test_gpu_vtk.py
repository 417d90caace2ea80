"""The reference's own sample DEM particle data (tests/golden/vtk, via rt_vtk_*) through the HIP path:
demo scene + VTK particles merged as main() does with LOAD_VTK (Main.cu:109-115).  The strips hold
~80 % index-degenerate triangles, so this exercises the |det| < 1e-6 rejection at scale."""
import os

import numpy as np
import pytest

from rtamd import Renderer
from rtamd.vtk import VtkSeriesPlayer, vtk_scene

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
VTK_DIR = os.path.join(HERE, "golden", "vtk")
F0 = os.path.join(VTK_DIR, "particle_000000000000000.vtk")
F1 = os.path.join(VTK_DIR, "particle_000000000000100.vtk")
SERIES = os.path.join(VTK_DIR, "particle_mesh.vtk.series")
THREADS = 16


def frac_within(a, b, lsb=1):
    d = np.abs(a.astype(np.int32) - b.astype(np.int32)).max(axis=-1)
    return float((d <= lsb).mean()), int(d.max())


@pytest.mark.parametrize("depth", [2, 10])
def test_vtk_scene_exact_parity(gpu_lib, depth):
    from oracle.oracle import OracleScene
    s = vtk_scene(SERIES)
    r = Renderer(s).build_acceleration_structure(5).configure_camera(240, 160, ray_trace_depth=depth)
    o = OracleScene(s, build_seed=5)
    o.camera(240, 160, ray_trace_depth=depth)
    for frame in (0, 21):
        o.update(frame)
        orgb, orgba, ocnt = o.render(threads=THREADS)
        rgba, rgb, st = r.render(frame, exact=True, want_rgb=True, count_work=True)
        assert (rgb != orgb).any(axis=2).sum() == 0, (frame, float(np.abs(rgb - orgb).max()))
        assert frac_within(rgba, orgba)[0] == 1.0
        for k in ("rays", "instance_visits", "triangle_tests", "sphere_quad_tests"):
            assert st[k] == ocnt[k], (frame, k)


@pytest.mark.parametrize("mode", ["sah", "lbvh"])
def test_vtk_scene_fast_modes_within_tolerance(gpu_lib, mode):
    from oracle.oracle import OracleScene
    s = vtk_scene(F0)
    r = Renderer(s).build_acceleration_structure(0, mode=mode).configure_camera(320, 180, ray_trace_depth=2)
    o = OracleScene(s, build_seed=0)
    o.camera(320, 180, ray_trace_depth=2)
    _, orgba, _ = o.render(threads=THREADS)
    rgba, _, _ = r.render(0)
    f, mx = frac_within(rgba, orgba)
    assert f >= 0.999, (mode, f, mx)


def test_series_playback_equals_fresh_scene(gpu_lib):
    """Loading series frame 1 into a running LBVH scene (triangles + instance bounds replaced, BLASes
    rebuilt on the GPU) renders the same bytes as a scene created from that file."""
    from oracle.oracle import OracleScene
    r = Renderer(vtk_scene(SERIES)).build_acceleration_structure(0, mode="lbvh").configure_camera(256, 144, ray_trace_depth=2)
    first = r.render(0, want_rgb=True)[1]
    player = VtkSeriesPlayer(r, SERIES)
    assert len(player) == 2 and player.load(1) == pytest.approx(0.01)
    played = r.render(0, want_rgb=True)[1]
    assert not np.array_equal(first, played)
    s1 = vtk_scene(F1)
    fresh = Renderer(s1).build_acceleration_structure(0, mode="lbvh").configure_camera(256, 144, ray_trace_depth=2)
    assert np.array_equal(played, fresh.render(0, want_rgb=True)[1])
    o = OracleScene(s1, build_seed=0)
    o.camera(256, 144, ray_trace_depth=2)
    _, orgba, _ = o.render(threads=THREADS)
    f, mx = frac_within(r.render(0)[0], orgba)
    assert f >= 0.999, (f, mx)
