"""Host scene preparation pinned against the reference's own known answers.

The counts below were produced by the reference's compiled host code
(Utils/obj_loader.h + Utils/BVH.h, identity transforms) — SURVEY.md §8(c):
  clock.obj       8265 tris / 3010 nodes (incl. dummy) / 1505 leaves / max depth 15
                  root AABB (-0.2619,-0.2181,0.3313)-(0.6082,0.8734,0.9389)
  table.obj       5184 / 2078 / 1039 leaves / depth 17
  table+clock    13449 / 5098
plus the readObj normalisation quirk (obj_loader.h:51-52): clock divided by
0.160946 instead of its true max extent 0.175673.
"""
import os

import numpy as np
import pytest

from ptsvgf.scene import ASSETS, SceneBuilder, build_scene, env_map, gen_cornell, gen_plant, gen_teapot, hdr_cache
from ptsvgf.scene import material, transform

CLOCK = os.path.join(ASSETS, "clock.obj")
TABLE = os.path.join(ASSETS, "table.obj")


def _build(paths):
    b = SceneBuilder()
    for i, p in enumerate(paths):
        b.add_obj(p, material(), transform(), True, i)
    b.build(8)
    return b


def test_clock_kat():
    b = _build([CLOCK])
    c = b.counts()
    assert (c["triangles"], c["nodes"], c["leaves"], c["max_depth"], c["max_leaf"]) == (8265, 3010, 1505, 15, 8)
    aabb = b.root_aabb()
    np.testing.assert_allclose(aabb, [-0.2619, -0.2181, 0.3313, 0.6082, 0.8734, 0.9389], atol=1e-4)


def test_table_kat():
    c = _build([TABLE]).counts()
    assert (c["triangles"], c["nodes"], c["leaves"], c["max_depth"]) == (5184, 2078, 1039, 17)


def test_table_clock_kat():
    c = _build([TABLE, CLOCK]).counts()
    assert (c["triangles"], c["nodes"]) == (13449, 5098)


def test_readobj_normalisation_quirk():
    """obj_loader.h:51-52 takes the y/z bounds against maxx/minx: divisor 0.160946, not 0.175673."""
    b = SceneBuilder()
    b.add_obj(CLOCK, material(), transform(), True, 0)
    b.build(8)
    _, _, raster = b.encode()  # the raster list keeps readObj's face order (pre-BVH sort)
    first = raster[:3]  # vertex 1 of face 1 ("f 1/1/1 ..."): raw (0.025443, -0.022332, 0.071237)
    np.testing.assert_allclose(first * np.float32(0.160946), [0.025443, -0.022332, 0.071237], rtol=2e-5)


def test_bvh_structure_invariants():
    b = _build([TABLE, CLOCK])
    tri, node, _ = b.encode()
    assert node[0, 0] == 255 and node[0, 1] == 128 and node[0, 3] == 30  # dummy node 0, main.cpp:88-94
    n = node.shape[0]
    covered = np.zeros(tri.shape[0], np.int32)
    stack = [(1, 0)]
    while stack:
        i, d = stack.pop()
        left, right, cnt, idx = int(node[i, 0]), int(node[i, 1]), int(node[i, 3]), int(node[i, 4])
        lo, hi = node[i, 6:9], node[i, 9:12]
        if cnt > 0:
            assert cnt <= 8
            covered[idx:idx + cnt] += 1
            p = tri[idx:idx + cnt, 0:9].reshape(-1, 3, 3)
            assert (p >= lo - 1e-7).all() and (p <= hi + 1e-7).all()
            continue
        for c in (left, right):
            assert 0 < c < n
            assert (node[c, 6:9] >= lo).all() and (node[c, 9:12] <= hi).all()
            stack.append((c, d + 1))
    assert (covered == 1).all(), "every triangle in exactly one leaf"


def test_encoding_layout():
    b = SceneBuilder()
    m = material(baseColor=(0.1, 0.2, 0.3), emissive=(1, 2, 3), subsurface=0.4, metallic=0.5, specular=0.6,
                 specularTint=0.7, roughness=0.8, anisotropic=0.9, sheen=0.11, sheenTint=0.12, clearcoat=0.13,
                 clearcoatGloss=0.14, IOR=1.5, transmission=0.16)
    b.add_obj(TABLE, m, transform(), True, 7)
    b.build(8)
    tri, _, _ = b.encode()
    t = tri[0]
    np.testing.assert_array_equal(t[18:21], np.float32([1, 2, 3]))            # emissive (Triangle.h:16)
    np.testing.assert_array_equal(t[21:24], np.float32([0.1, 0.2, 0.3]))      # baseColor
    np.testing.assert_array_equal(t[24:27], np.float32([0.4, 0.5, 0.6]))      # param1 (main.cpp:116)
    np.testing.assert_array_equal(t[27:30], np.float32([0.7, 0.8, 0.9]))      # param2
    np.testing.assert_array_equal(t[30:33], np.float32([0.11, 0.12, 0.13]))   # param3
    np.testing.assert_array_equal(t[33:36], np.float32([0.14, 1.5, 0.16]))    # param4
    assert t[42] == 7.0 and t[43] == 0.0                                       # objIndex (main.cpp:123)
    nrm = tri[:, 9:18].reshape(-1, 3, 3)
    np.testing.assert_allclose(np.linalg.norm(nrm, axis=-1), 1.0, atol=1e-5)  # smooth normals normalised


def test_hdr_cache_properties():
    hdr = env_map(128, 64)
    cache = hdr_cache(hdr)
    assert cache.shape == hdr.shape
    np.testing.assert_allclose(cache[..., 2].sum(), 1.0, rtol=1e-3)  # B = normalised luminance pdf
    assert (cache[..., 0] >= 0).all() and (cache[..., 0] < 1).all()
    assert (cache[..., 1] >= 0).all() and (cache[..., 1] < 1).all()
    lum = 0.2 * hdr[..., 0] + 0.7 * hdr[..., 1] + 0.1 * hdr[..., 2]
    np.testing.assert_allclose(cache[..., 2], lum / lum.sum(), rtol=1e-4, atol=1e-9)


def test_hdr_cache_single_bright_texel():
    """A one-hot environment makes every cache entry sample that texel (hdr_compute.h:71-86)."""
    hdr = np.full((16, 32, 3), 1e-6, np.float32)
    hdr[5, 9] = 1000.0
    cache = hdr_cache(hdr)
    xs = np.round(cache[..., 0] * 32).astype(int)
    ys = np.round(cache[..., 1] * 16).astype(int)
    # xi == 0 exactly (row 0 / column 0) lower_bounds to entry 0; every other entry finds the texel
    assert (xs[1:, :] == 9).all() and (ys[1:, 1:] == 5).all()


def test_generators_deterministic():
    a, b = gen_plant(0, 30), gen_plant(0, 30)
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])
    assert not np.array_equal(gen_plant(1, 30)[0], a[0])
    p, i = gen_teapot(32)
    assert i.max() < p.shape[0] and p.shape[0] > 100
    p, i = gen_cornell()
    assert i.shape == (10, 3)


@pytest.mark.parametrize("name", ["clock", "table_clock_plant", "cornell_teapot"])
def test_named_scenes_build(name):
    s = build_scene(name, hdr_size=(64, 32), plant_leaves=10)
    assert s.tri_enc.shape[1] == 45 and s.node_enc.shape[1] == 12
    assert s.raster.size == s.ntris * 18
    assert s.counts["max_depth"] < 32  # the GPU traversal stack (pt_device.h kStack)
