"""CPU checks of tests/lbvh_ref.py, the restatement that GPU-built (RT_BUILD_LBVH) trees are compared
with in test_gpu_lbvh.py: Morton codes, the radix-tree split, leaf collapse and tree invariants."""
import numpy as np

from lbvh_ref import check_tree, lbvh_tree, morton_codes


def _boxes_around(c, half=0.01):
    c = np.asarray(c, np.float32)
    b = np.empty((c.shape[0], 6), np.float32)
    b[:, 0::2] = c - np.float32(half)
    b[:, 1::2] = c + np.float32(half)
    return b


def test_morton_interleaves_xyz():
    c = np.array([[0, 0, 0], [1, 1, 1], [1, 0, 0], [0, 1, 0], [0, 0, 1]], np.float32)
    m = morton_codes(c)
    assert m[0] == 0
    assert m[1] == (1 << 30) - 1                      # 1023 in every axis
    assert m[2] == 0b100100100100100100100100100100   # x bits at 3k + 2
    assert m[3] == m[2] >> 1 and m[4] == m[2] >> 2


def test_morton_flat_axis_quantises_to_zero():
    c = np.array([[0, 5, 0], [1, 5, 1], [0.5, 5, 0.25]], np.float32)
    m = morton_codes(c)
    assert all(int(x) & 0b010010010010010010010010010010 == 0 for x in m)   # y bits all zero


def test_two_clusters_split_at_root():
    rng = np.random.default_rng(1)
    a = rng.uniform(0.0, 0.1, (10, 3))
    b = rng.uniform(0.9, 1.0, (7, 3))
    c = np.concatenate([a, b]).astype(np.float32)
    nb, ci, refs = lbvh_tree(_boxes_around(c), c, 4)
    left, right = int(ci[0, 1]), int(ci[0, 1]) + 1

    def items(j):
        if ci[j, 0]:
            return set(refs[ci[j, 1]:ci[j, 1] + ci[j, 0]].tolist())
        k = int(ci[j, 1])
        return items(k) | items(k + 1)
    assert items(left) == set(range(10)) and items(right) == set(range(10, 17))


def test_identical_centroids_still_split_by_position():
    c = np.zeros((9, 3), np.float32)
    nb, ci, refs = lbvh_tree(_boxes_around(c), c, 2)
    assert refs.tolist() == list(range(9))            # stable order, split by index bits
    check_tree(nb, ci, refs, _boxes_around(c), 2)


def test_small_sets_are_one_leaf():
    for n, cap in ((1, 4), (3, 4), (4, 4), (2, 2)):
        c = np.random.default_rng(n).uniform(0, 1, (n, 3)).astype(np.float32)
        nb, ci, refs = lbvh_tree(_boxes_around(c), c, cap)
        assert nb.shape[0] == 1 and ci[0, 0] == n


def test_random_trees_are_valid():
    rng = np.random.default_rng(7)
    for n in (5, 64, 1000):
        c = rng.normal(size=(n, 3)).astype(np.float32)
        b = _boxes_around(c, 0.05)
        nb, ci, refs = lbvh_tree(b, c, 4)
        h = check_tree(nb, ci, refs, b, 4)
        assert h <= 40
        assert int((ci[:, 0] == 0).sum()) + 1 == int((ci[:, 0] > 0).sum())   # binary: leaves = interior + 1
