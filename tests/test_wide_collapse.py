"""CPU check of the BVH2 -> BVH4 collapse (csrc/bvh_build.hpp flatten_tree_wide, option "wide"), in both forms —
two binary levels per quad (halves: the reference's trees, visited in its pair order) and the greedy collapse (host
SAH trees): the quad form holds exactly the binary tree's leaves, every quad child box (and with halves every half's
union box) is a node box of the binary tree, quads hold 2-4 children, and the tree is about half as deep."""
import json
import os
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def checker(tmp_path_factory):
    exe = str(tmp_path_factory.mktemp("wide") / "wide_collapse_check")
    subprocess.run(["g++", "-std=c++17", "-O1", "-D__host__=", "-D__device__=", "-o", exe,
                    os.path.join(HERE, "cpp", "wide_collapse_check.cpp")], check=True)
    return exe


@pytest.mark.parametrize("halves", [1, 0])
@pytest.mark.parametrize("n,sah", [(1, 1), (3, 1), (5, 0), (17, 1), (1000, 1), (1000, 0), (20000, 1)])
def test_quad_form_preserves_leaves_and_boxes(checker, n, sah, halves):
    r = json.loads(subprocess.run([checker, str(n), str(sah), str(halves)], check=True, capture_output=True,
                                  text=True).stdout)
    assert r["slots_equal"] == 1 and r["bad_boxes"] == 0, r
    if r["quads"]:
        assert 2 <= r["min_children"] <= 4 and r["mean_children"] > 3.0 or n < 20, r
        assert r["height4"] <= (r["height2"] + 1) // 2 + 2, r
        assert r["quads"] <= r["pairs"], r
