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
    fast, _, _ = r.render(frame)
    d = np.abs(fast[y0:y0 + h, x0:x0 + w].astype(int) - vec[f"img_{name}_rgba"].astype(int)).max(axis=2)
    assert (d <= 1).mean() >= 0.995
