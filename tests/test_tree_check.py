"""The trees the library derives from the reference tree (capi.hip build_anyhit_tree: SAH tree over the reference
leaves, treelet restructuring, fine leaves, 4-wide collapse greedy or by dynamic program), checked on the host through
pt_tree_check (no device): the properties every walk's result preservation rests on (DESIGN.md "Closest-hit rays on
the SAH tree", "The traversal in round 6"):
  * every triangle of a reference leaf is held by exactly one leaf of each tree, and no other triangle is;
  * every child box lies inside its parent's box, and every leaf box holds its triangles (under a reference leaf's own
    box the fine boxes only cull: there each leaf box must hold its triangles instead);
  * the treelet passes do not raise the SAH cost, and the dynamic program does not raise the summed 4-wide node area.
The walks' bits on the GPU are the parity tests' (test_wide_tree_is_result_preserving, test_gpu_fullsize)."""
import ctypes as C

import numpy as np
import pytest

from ptsvgf._lib import pt

N = 12  # PT_TREE_CHECK_COUNT


def check(scene, collapse, treelet):
    lib = pt()
    node = np.ascontiguousarray(scene.node_enc, np.float32)
    tri = np.ascontiguousarray(scene.tri_enc, np.float32)
    out = (C.c_double * N)()
    rc = lib.pt_tree_check(node.ctypes.data_as(C.POINTER(C.c_float)), node.shape[0],
                           tri.ctypes.data_as(C.POINTER(C.c_float)), tri.shape[0], collapse, treelet, out, N)
    assert rc == 0, lib.pt_last_error()
    keys = ("binary_ok", "anyhit4_ok", "closest4_ok", "contain_ok", "sah_before", "sah_after", "area_anyhit",
            "area_closest", "wide_nodes", "depth", "need4", "two_trees")
    return dict(zip(keys, list(out)))


@pytest.mark.parametrize("scene_name", ["scene_small", "scene_cornell", "scene_nan", "scene_bench"])
def test_trees_hold_the_reference_leaves(scene_name, request):
    scene = request.getfixturevalue(scene_name)
    res = {}
    for collapse in (0, 1, 2, 3):
        for treelet in (0, 1, 3):
            r = check(scene, collapse, treelet)
            res[collapse, treelet] = r
            assert r["binary_ok"] == 1 and r["anyhit4_ok"] == 1 and r["closest4_ok"] == 1, (collapse, treelet, r)
            assert r["contain_ok"] == 1, (collapse, treelet, r)
            assert r["sah_after"] <= r["sah_before"] * (1 + 1e-9), r
            assert r["two_trees"] == (1 if collapse in (2, 3) and r["wide_nodes"] > 1 else 0) or r["wide_nodes"] <= 1
            assert r["depth"] < 32, r  # kStack: the binary walks' stack
    for treelet in (0, 1, 3):
        greedy, dp = res[0, treelet], res[1, treelet]
        # the dynamic program minimises exactly the summed node area the greedy grouping also reports
        assert dp["area_anyhit"] <= greedy["area_anyhit"] * (1 + 1e-6), (greedy, dp)
        # mode 2: the any-hit tree is the program's, the closest-hit tree the greedy one; mode 3 the reverse
        assert res[2, treelet]["area_anyhit"] == pytest.approx(dp["area_anyhit"])
        assert res[2, treelet]["area_closest"] == pytest.approx(greedy["area_anyhit"])
        assert res[3, treelet]["area_anyhit"] == pytest.approx(greedy["area_anyhit"])
        assert res[3, treelet]["area_closest"] == pytest.approx(dp["area_anyhit"])


def test_tree_check_rejects_bad_arguments(scene_small):
    lib = pt()
    node = np.ascontiguousarray(scene_small.node_enc, np.float32)
    tri = np.ascontiguousarray(scene_small.tri_enc, np.float32)
    out = (C.c_double * N)()
    fp = C.POINTER(C.c_float)
    args = (node.ctypes.data_as(fp), node.shape[0], tri.ctypes.data_as(fp), tri.shape[0])
    assert lib.pt_tree_check(*args, 0, 1, out, N - 1) == -6  # PT_ERR_ARG: output too short
    assert lib.pt_tree_check(*args, 4, 1, out, N) == -6      # no collapse mode 4
    assert lib.pt_tree_check(*args, 0, -1, out, N) == -6
    bad = node.copy()
    bad[bad[:, 3] > 0, 3] = 16  # a leaf of 16 triangles: more than a leaf ref holds
    assert lib.pt_tree_check(bad.ctypes.data_as(fp), bad.shape[0], *args[2:], 0, 1, out, N) == -7  # PT_ERR_FORMAT


def test_tree_check_finds_a_box_that_misses_its_triangles(scene_small):
    """The checker is not vacuous: a reference leaf whose box is shrunk so that it no longer holds its triangles (a
    tree the reference's own walk would also get wrong) is reported."""
    node = np.array(scene_small.node_enc, np.float32)
    leaves = np.nonzero((node[:, 3] > 0) & (node[:, 3] <= 4))[0]
    i = int(leaves[len(leaves) // 2])
    lo, hi = node[i, 6:9].copy(), node[i, 9:12].copy()
    node[i, 9:12] = lo + 0.25 * (hi - lo)
    scene = type("S", (), {"node_enc": node, "tri_enc": scene_small.tri_enc})
    assert check(scene, 2, 1)["contain_ok"] == 0
    assert check(scene_small, 2, 1)["contain_ok"] == 1
