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


@pytest.mark.parametrize("leaf_n", [1, 4, 8, 15])
def test_oracle_tree_valid_on_scene(scene_small, leaf_n):
    tri, nodes = L.lbvh(scene_small.tri_enc, leaf_n)
    info = L.check_tree(tri, nodes, leaf_n)
    assert info["depth"] < 256  # the reference walk's stack (path_tracing.frag:378)
    # a permutation of the input records
    a = np.sort(scene_small.tri_enc.view(np.uint32), axis=0)
    assert np.array_equal(np.sort(tri.view(np.uint32), axis=0), a)
    print(f"leaf_n {leaf_n}: {len(nodes)} nodes, {info['leaves']} leaves, depth {info['depth']}")


@pytest.mark.parametrize("n", [1, 2, 3, 17, 256, 1000])
@pytest.mark.parametrize("flat", [None, 1])
def test_oracle_tree_valid_small(n, flat):
    t = _random_tris(n, seed=n, flat_axis=flat)
    tri, nodes = L.lbvh(t, 4)
    L.check_tree(tri, nodes, 4)
    assert sorted(tri[:, 42].astype(int)) == list(range(n))
    k, b = L.keys(t)
    assert len(np.unique(k)) == n and (1 << b) >= n
    assert np.array_equal(nodes[0], L.DUMMY_NODE)


def test_oracle_leaf_order_follows_morton_keys():
    t = _random_tris(500, seed=3)
    tri, _ = L.lbvh(t, 8)
    k, b = L.keys(t)
    assert np.array_equal(tri[:, 42].astype(np.int64), (np.sort(k) & np.uint64((1 << b) - 1)).astype(np.int64))
