"""Scene generators: the demo scene restatement and the synthetic VTK stand-in."""
import numpy as np

from rtamd import abi, scenes


def test_demo_scene_matches_main_cu():
    s = scenes.demo_scene()
    assert len(s.spheres) == 2 and len(s.parallelograms) == 1 and s.triangle_count == 1
    assert len(s.roughs) == 4 and len(s.metals) == 1
    assert [(d["type"], d["index"]) for d in s.instances] == [(0, 0), (0, 1), (1, 0), (2, 0), (0, 1)]
    assert s.camera["fov"] == 90.0 and s.camera["ray_trace_depth"] == 10


def test_uv_sphere_is_closed_manifold():
    v, f = scenes.uv_sphere_template(1024)
    assert f.shape == (1024, 3)
    edges = {}
    for tri in f:
        for a, b in ((tri[0], tri[1]), (tri[1], tri[2]), (tri[2], tri[0])):
            edges[(min(a, b), max(a, b))] = edges.get((min(a, b), max(a, b)), 0) + 1
    assert set(edges.values()) == {2}
    # outward winding: face normal points away from the centre
    p = v[f]
    n = np.cross(p[:, 1] - p[:, 0], p[:, 2] - p[:, 0])
    assert (np.einsum("ij,ij->i", n, p.mean(axis=1)) > 0).all()


def test_synth_particles_counts_and_placement():
    tris, inst = scenes.synth_particles(5, 1024, seed=1)
    assert tris.shape == (5 * 1024,) and len(inst) == 5
    assert (tris["material_type"] == abi.METAL).all() and (tris["has_normals"] == 1).all()
    for d in inst:
        lo = np.asarray(d["bounds"][0::2]); hi = np.asarray(d["bounds"][1::2])
        assert (lo >= [-0.48 - 0.061, -0.48 - 0.061, 0.34 - 0.061]).all()
        assert (hi <= [0.46 + 0.061, 0.46 + 0.061, 0.47 + 0.061]).all()
        assert d["shift"] == (0.0, 4.0, 0.0) and d["rotate"] == (90.0, 0.0, 0.0)
    n = np.linalg.norm(tris["normal"], axis=2)
    assert np.allclose(n, 1.0, atol=1e-6)


def test_particles_prepended_like_vtk_merge():
    s = scenes.demo_with_particles(3, 1024)
    assert s.triangle_count == 3 * 1024 + 1
    tri_inst = [d for d in s.instances[:5] if d["type"] == abi.TRIANGLE][0]
    assert tri_inst["index"] == 3 * 1024                  # Renderer.cu:106-108
    assert [d["index"] for d in s.instances[5:]] == [0, 1024, 2048]


def test_config_table():
    c2 = scenes.CONFIGS["C2"]
    assert (c2.width, c2.height, c2.spp, c2.depth, c2.particles * 1024) == (1920, 1080, 1, 2, 69632)
    c3 = scenes.CONFIGS["C3"]
    assert c3.particles * 1024 == 260096 and c3.spp == 4 and c3.depth == 4
    c5 = scenes.CONFIGS["C5"]
    assert c5.particles * 1024 >= 10_000_000 and (c5.width, c5.height) == (3840, 2160)


def test_scene_desc_marshalling():
    s = scenes.demo_with_particles(2, 1024)
    d = s.desc()
    assert d.triangle_count == 2049 and d.instance_count == 7
    assert d.triangles[0].has_normals == 1 and d.triangles[2048].has_normals == 0
    assert d.instances[6].has_local_bounds == 1 and d.instances[6].primitive_count == 1024
