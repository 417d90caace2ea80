"""The oracle reproduces the committed golden fixtures bit for bit (tests/golden/make_golden.py).

The fixtures freeze the oracle (the reference restatement) against accidental change; the GPU
tests (test_gpu_golden.py) check the HIP path against the same vectors without the oracle."""
import os
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = os.path.join(HERE, "golden")
sys.path.insert(0, GOLDEN)


@pytest.fixture(scope="module")
def fresh(oracle_lib):
    import make_golden
    return make_golden.prim_kats(), make_golden.hits_and_images()


def test_prim_kats_reproduce(fresh):
    g = np.load(os.path.join(GOLDEN, "prim_kats.npz"))
    kats, _ = fresh
    assert set(g.files) == set(kats)
    for k in g.files:
        assert np.array_equal(g[k], kats[k], equal_nan=True), k
    # sanity: the KAT sets exercise both outcomes
    for k in ("sphere", "quad", "tri"):
        hit = g[f"{k}_out"][:, 0]
        assert 0.05 < hit.mean() < 0.95, k
    assert 0.05 < g["aabb_out"][:, 0].mean() < 0.95


def test_scene_vectors_reproduce(fresh):
    g = np.load(os.path.join(GOLDEN, "scene_vectors.npz"))
    _, vec = fresh
    assert set(g.files) == set(vec)
    for k in g.files:
        assert np.array_equal(g[k], vec[k], equal_nan=True), k
