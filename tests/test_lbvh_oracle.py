"""The LBVH restatement (oracle/lbvh_ref.py), the checker of the GPU builder pt_bvh_build: on the reference's
own scenes and on tiny and degenerate inputs its trees are valid BVHs in the reference's node format (every
triangle in one leaf, leaves of <= leaf_n, boxes the exact glm min/max of what they hold, root at node 1), its keys
are unique and sorted, and it keeps the triangle records intact (a permutation)."""
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
import lbvh_ref as L  # noqa: E402


def _random_tris(n, seed=0, flat_axis=None):
    rng = np.random.default_rng(seed)
    t = np.zeros((n, 45), np.float32)
    t[:, :9] = rng.uniform(-1, 1, (n, 9)).astype(np.float32)
    if flat_axis is not None:
        t[:, flat_axis:9:3] = 0.5  # every vertex on one plane: a zero-extent centroid axis
    t[:, 42] = np.arange(n)  # objIndex: identifies the record after reordering
    return t


@pytest.mark.parametrize("ploc", [0, 16])
@pytest.mark.parametrize("leaf_n", [1, 4, 8, 15])
def test_oracle_tree_valid_on_scene(scene_small, leaf_n, ploc):
    tri, nodes = L.lbvh(scene_small.tri_enc, leaf_n, ploc)
    info = L.check_tree(tri, nodes, leaf_n)
    assert info["depth"] < 256  # the reference walk's stack (path_tracing.frag:378)
    # a permutation of the input records
    a = np.sort(scene_small.tri_enc.view(np.uint32), axis=0)
    assert np.array_equal(np.sort(tri.view(np.uint32), axis=0), a)
    print(f"leaf_n {leaf_n} ploc {ploc}: {len(nodes)} nodes, {info['leaves']} leaves, depth {info['depth']}")


@pytest.mark.parametrize("ploc", [0, 1, 16])
@pytest.mark.parametrize("n", [1, 2, 3, 17, 256, 1000])
@pytest.mark.parametrize("flat", [None, 1])
def test_oracle_tree_valid_small(n, flat, ploc):
    t = _random_tris(n, seed=n, flat_axis=flat)
    tri, nodes = L.lbvh(t, 4, ploc)
    L.check_tree(tri, nodes, 4)
    assert sorted(tri[:, 42].astype(int)) == list(range(n))
    k, b = L.keys(t)
    assert len(np.unique(k)) == n and (1 << b) >= n
    assert np.array_equal(nodes[0], L.DUMMY_NODE)


def test_ploc_top_lowers_the_surface_area_cost(scene_small):
    """PLOC's top is a surface-area-driven clustering: its SAH-style cost (sum of interior half areas) is below the
    LBVH's over the same leaves."""
    def cost(nodes):
        d = nodes[1:, 9:12] - nodes[1:, 6:9]
        a = (d[:, 0] * d[:, 1] + d[:, 1] * d[:, 2]) + d[:, 2] * d[:, 0]
        return float(a[nodes[1:, 3] == 0].astype(np.float64).sum())
    _, lb = L.lbvh(scene_small.tri_enc, 8, 0)
    _, pl = L.lbvh(scene_small.tri_enc, 8, 16)
    assert len(lb) == len(pl) and cost(pl) < cost(lb)
    print(f"interior half-area sum: LBVH {cost(lb):.1f}, PLOC {cost(pl):.1f}")


def test_oracle_leaf_order_follows_morton_keys():
    t = _random_tris(500, seed=3)
    tri, _ = L.lbvh(t, 8)
    k, b = L.keys(t)
    assert np.array_equal(tri[:, 42].astype(np.int64), (np.sort(k) & np.uint64((1 << b) - 1)).astype(np.int64))


@pytest.mark.parametrize("ploc", [0, 16])
def test_oracle_nan_vertices(ploc):
    """NaN vertex positions (garbage input) still give a valid tree: NaN centroids stay out of the bounds and fall
    in Morton cell 0, and PLOC ranks NaN boxes last, so it terminates."""
    t = _random_tris(300, seed=9)
    t[[5, 77, 150], 0] = np.nan
    tri, nodes = L.lbvh(t, 4, ploc)
    L.check_tree(tri, nodes, 4)
    assert sorted(tri[:, 42].astype(int)) == list(range(300))
