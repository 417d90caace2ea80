"""Scene ingestion: rt_vtk_* against an independent numpy parser of the
reference's own sample particle files (tests/golden/vtk), host-only (no GPU)."""
import os

import numpy as np
import pytest

import vtk_ref
from rtamd import abi, scenes
from rtamd.vtk import VtkFile, read_series, vtk_scene

HERE = os.path.dirname(os.path.abspath(__file__))
VTK_DIR = os.path.join(HERE, "golden", "vtk")
F0 = os.path.join(VTK_DIR, "particle_000000000000000.vtk")
F1 = os.path.join(VTK_DIR, "particle_000000000000100.vtk")
SERIES = os.path.join(VTK_DIR, "particle_mesh.vtk.series")


@pytest.fixture(scope="module")
def lib(rtlib_path):
    return abi.load_library()


@pytest.mark.parametrize("path", [F0, F1])
def test_counts_and_particles_match_independent_parser(lib, path):
    pts, strips, ids, vel = vtk_ref.parse(path)
    f = VtkFile(path)
    assert f.point_count == pts.shape[0] == 3200
    assert f.particle_count == len(strips) == 25
    assert f.strip_vertex_count == sum(len(s) for s in strips)
    assert f.triangle_count == sum(len(s) - 2 for s in strips)
    got = f.particles()
    want = vtk_ref.particles(pts, strips, ids, vel)
    for g, w in zip(got, want):
        assert int(g["id"]) == w["id"]
        assert np.array_equal(g["velocity"], w["velocity"])
        assert np.array_equal(g["bounds"], w["bounds"])
        assert np.array_equal(g["centroid"], w["centroid"])
        assert int(g["vertex_count"]) == w["vertex_count"]


def test_convert_triangles_and_instances(lib):
    pts, strips, ids, vel = vtk_ref.parse(F0)
    tris, inst = VtkFile(F0).convert(7)
    assert np.array_equal(tris["vertex"], vtk_ref.triangles(pts, strips))
    assert (tris["material_type"] == abi.METAL).all() and (tris["material_index"] == 0).all()
    assert (tris["has_normals"] == 1).all()
    want = vtk_ref.particles(pts, strips, ids, vel)
    first = 7
    for d, w, st in zip(inst, want, strips):
        assert d["type"] == abi.TRIANGLE and d["index"] == first and d["count"] == len(st) - 2
        assert np.array_equal(np.asarray(d["bounds"], np.float32), w["bounds"])
        assert np.array_equal(np.asarray(d["centroid"], np.float32), w["centroid"])
        assert d["shift"] == (0.0, 4.0, 0.0) and d["rotate"] == (90.0, 0.0, 0.0) and d["scale"] == (3.0, 3.0, 3.0)
        first += len(st) - 2


def test_normals_unit_and_outward(lib):
    """Restated vtkPolyDataNormals (parity unpinned): unit vertex normals pointing away from each
    particle's centroid on (nearly) every vertex of these convex particles."""
    f = VtkFile(F0)
    pos, nrm = f.vertices()
    lens = np.linalg.norm(nrm, axis=1)
    assert np.allclose(lens, 1.0, atol=1e-5)
    parts = f.particles()
    out = np.zeros(len(pos), bool)
    for p in parts:
        a, b = int(p["first_vertex"]), int(p["first_vertex"] + p["vertex_count"])
        out[a:b] = ((pos[a:b] - p["centroid"]) * nrm[a:b]).sum(axis=1) > 0
    assert out.mean() >= 0.99


def test_series_index(lib):
    entries = read_series(SERIES)
    assert [os.path.basename(p) for p, _ in entries] == [os.path.basename(F0), os.path.basename(F1)]
    assert [t for _, t in entries] == [0.0, np.float32(0.01)]
    assert all(os.path.exists(p) for p, _ in entries)


def test_vtk_scene_merges_like_load_vtk(lib):
    s = vtk_scene(SERIES)
    n = VtkFile(F0).triangle_count
    assert s.triangle_count == n + 1
    assert len(s.instances) == 5 + 25
    assert [d["index"] for d in s.instances if d["type"] == abi.TRIANGLE][0] == n      # demo triangle shifted
    scenes.Scene.desc(s)                                                                # marshals


def test_errors_are_reported(lib, tmp_path):
    bad = tmp_path / "bad.vtk"
    bad.write_bytes(b"not a vtk file\n")
    with pytest.raises(abi.RtError, match="header"):
        VtkFile(str(bad))
    poly = tmp_path / "poly.vtk"
    poly.write_text("# vtk DataFile Version 2.0\nx\nASCII\nDATASET POLYDATA\nPOINTS 3 float\n0 0 0 1 0 0 0 1 0\n"
                    "POLYGONS 1 4\n3 0 1 2\n")
    with pytest.raises(abi.RtError, match="illegal cell type"):
        VtkFile(str(poly))
    with pytest.raises(abi.RtError):
        VtkFile(str(tmp_path / "missing.vtk"))


def test_ascii_file_with_field_arrays(lib, tmp_path):
    p = tmp_path / "a.vtk"
    p.write_text("# vtk DataFile Version 3.0\nascii strip\nASCII\nDATASET POLYDATA\nPOINTS 4 float\n"
                 "0 0 0  1 0 0  0 1 0  1 1 0\nTRIANGLE_STRIPS 1 5\n4 0 1 2 3\n"
                 "CELL_DATA 1\nFIELD FieldData 2\nid 1 1 int\n42\nvel 3 1 double\n1 2 3\n")
    f = VtkFile(str(p))
    assert f.triangle_count == 2
    part = f.particles()[0]
    assert int(part["id"]) == 42 and part["velocity"].tolist() == [1.0, 2.0, 3.0]
    tris, inst = f.convert(0)
    assert tris["vertex"][1].tolist() == [[1, 0, 0], [1, 1, 0], [0, 1, 0]]   # odd triangle: 2nd/3rd swapped


@pytest.mark.parametrize("body", [
    # 3 * n wraps to 2 in 64-bit arithmetic
    b"POINTS 6148914691236517206 float\n",
    # comps * tuples wraps to 0: a wrapped size used to pass and then index far out of bounds
    b"POINTS 3 float\n0 0 0 1 0 0 0 1 0\nTRIANGLE_STRIPS 1 4\n3 0 1 2\nCELL_DATA 4\n"
    b"FIELD FieldData 1\nid 4611686018427387904 4 int\n1\n",
    # a huge count that does not wrap must fail before allocating (no bad_alloc through the C ABI)
    b"POINTS 3 float\n0 0 0 1 0 0 0 1 0\nTRIANGLE_STRIPS 1 4\n3 0 1 2\nCELL_DATA 1\n"
    b"SCALARS id int 1000000000000000\n1\n",
    # negative / oversized strip length
    b"POINTS 3 float\n0 0 0 1 0 0 0 1 0\nTRIANGLE_STRIPS 1 4\n-5 0 1 2\n",
])
def test_hostile_counts_fail_cleanly(lib, tmp_path, body):
    """Counts from the file are untrusted: products are checked, sizes are bounded by the bytes left in
    the file before any allocation, and no C++ exception crosses the C ABI."""
    p = tmp_path / "hostile.vtk"
    p.write_bytes(b"# vtk DataFile Version 3.0\nx\nASCII\nDATASET POLYDATA\n" + body)
    with pytest.raises(abi.RtError):
        VtkFile(str(p))
