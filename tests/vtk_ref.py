"""Independent numpy parser of legacy BINARY VTK polydata particle files — TEST INFRASTRUCTURE ONLY,
the checker of rt_vtk_read / rt_vtk_convert (vtk_reader.cpp).  It reads exactly the layout the
reference's sample data uses (POINTS double, TRIANGLE_STRIPS, CELL_DATA SCALARS id int + VECTORS
vel double), big-endian, and restates VTKReader.cu:87-150 (id, velocity, bounds, centroid, strip
vertices) and :166-220 (strip -> triangles with odd triangles' vertices 2/3 swapped)."""
from __future__ import annotations

import numpy as np


def _section(data: bytes, kw: bytes, start: int = 0):
    i = data.index(kw, start)
    j = data.index(b"\n", i)
    return data[i:j].split(), j + 1


def parse(path: str):
    data = open(path, "rb").read()
    hdr, p = _section(data, b"POINTS")
    n, t = int(hdr[1]), hdr[2]
    assert t == b"double"
    pts = np.frombuffer(data, ">f8", 3 * n, p).reshape(n, 3)
    hdr, p = _section(data, b"TRIANGLE_STRIPS", p)
    cells, size = int(hdr[1]), int(hdr[2])
    lst = np.frombuffer(data, ">i4", size, p).astype(np.int64)
    strips, k = [], 0
    for _ in range(cells):
        m = int(lst[k])
        strips.append(lst[k + 1:k + 1 + m])
        k += m + 1
    hdr, p = _section(data, b"SCALARS id", p)
    _, p = _section(data, b"LOOKUP_TABLE", p)
    ids = np.frombuffer(data, ">i4", cells, p).astype(np.uint64)
    hdr, p = _section(data, b"VECTORS vel", p)
    vel = np.frombuffer(data, ">f8", 3 * cells, p).reshape(cells, 3)
    return pts, strips, ids, vel


def particles(pts, strips, ids, vel):
    out = []
    for s, st in enumerate(strips):
        v = pts[st]
        b = np.empty(6, np.float32)
        b[0::2] = v.min(axis=0).astype(np.float32)
        b[1::2] = v.max(axis=0).astype(np.float32)
        c = np.zeros(3)
        for q in v:                                  # double accumulation in strip order
            c += q
        out.append(dict(id=int(ids[s]), velocity=vel[s].astype(np.float32), bounds=b,
                        centroid=(c / len(st)).astype(np.float32), vertex_count=len(st)))
    return out


def triangles(pts, strips):
    """[T, 3, 3] float32 vertex positions of every strip triangle (odd ones swapped)."""
    out = []
    for st in strips:
        for j in range(len(st) - 2):
            a, b, c = (st[j], st[j + 1], st[j + 2]) if j % 2 == 0 else (st[j], st[j + 2], st[j + 1])
            out.append(pts[[a, b, c]])
    return np.asarray(out).astype(np.float32)
