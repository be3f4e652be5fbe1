"""CPU restatement of the GPU LBVH builder (path-tracing-svgf_amd/csrc/kernels_bvh.hip, pt_bvh_build).

TEST INFRASTRUCTURE ONLY: tests/ use it as the checker of the HIP builder; nothing in the product imports it.

Parity status: the reference has no GPU builder (it builds once on the host with buildBVHwithSAH,
Utils/BVH.h:42-173, restated bit-exactly in csrc/scene_prep.cpp and pinned by tests/test_scene_kat.py), so this
builder's tree is **parity unpinned** against the reference. What is pinned: the buffer formats are the reference's
(Triangle_encoded, Utils/Triangle.h:12-24; BVHNode_encoded, Utils/BVH.h:18-22, encoded as main.cpp:122-133 does,
dummy node 0 as main.cpp:88-94), and rendering over the built buffers is bit-exact against the oracle path tracer
walking the same buffers (tests/test_gpu_bvh.py).

Algorithm (Karras, HPG 2012, as published), with the kernel's float32 arithmetic:
  centroid  c = ((p1 + p2) + p3) / 3                         (cmpx's centre, BVH.h:25-29)
  cell      floor((c - lo) / (hi - lo) * 1024) clamped to [0, 1023] per axis (0 for a flat axis)
  key       morton30(x, y, z) << b | index,  b = bits of n - 1 (>= 1): unique keys
  tree      the binary radix tree of the sorted keys: node [f, l] splits after the last key sharing more than
            clz(k[f] ^ k[l]) leading bits with k[f]; its children are internal nodes gamma / gamma + 1 (Karras'
            numbering) or primitives
  boxes     primitive: glm min/max over its three vertices (BVH.h:54-66); internal: union of its two children
  leaves    a node whose range holds <= leaf_n primitives is a leaf (n = count, index = first sorted position)
  numbering reachable nodes in the order [internal 0 .. n-2, primitive 0 .. n-1], from node 1 (the root)
With ploc_radius > 0 the LBVH leaves are kept and the tree above them is PLOC's (ploc_top).
"""
from __future__ import annotations

import numpy as np

DUMMY_NODE = np.array([255, 128, 0, 30, 0, 0, 1, 1, 0, 0, 1, 0], np.float32)  # main.cpp:88-94


def _spread10(v: np.ndarray) -> np.ndarray:
    x = v.astype(np.uint64) & np.uint64(0x3FF)
    for sh, m in ((16, 0x030000FF), (8, 0x0300F00F), (4, 0x030C30C3), (2, 0x09249249)):
        x = (x | (x << np.uint64(sh))) & np.uint64(m)
    return x


def _gmin(a, b):  # glm::min(a, b) = b < a ? b : a
    return np.where(b < a, b, a)


def _gmax(a, b):  # glm::max(a, b) = a < b ? b : a
    return np.where(a < b, b, a)


def keys(tri_enc: np.ndarray):
    """Morton keys (uint64) of the triangles and the index bit count b."""
    t = np.asarray(tri_enc, np.float32).reshape(-1, 45)
    n = t.shape[0]
    c = ((t[:, 0:3] + t[:, 3:6]) + t[:, 6:9]) / np.float32(3.0)
    with np.errstate(invalid="ignore"), __import__("warnings").catch_warnings():
        __import__("warnings").simplefilter("ignore", RuntimeWarning)
        lo, hi = np.nanmin(c, axis=0), np.nanmax(c, axis=0)  # NaN centroids stay out of the bounds
    ext = (hi - lo).astype(np.float32)
    with np.errstate(divide="ignore", invalid="ignore"):
        q = np.where(ext > 0, (c - lo) / np.where(ext > 0, ext, np.float32(1)), np.float32(0)).astype(np.float32)
    v = np.floor(q * np.float32(1024.0))
    v = np.where(np.isnan(v), np.float32(0), v)  # NaN -> cell 0
    cell = np.clip(v, 0, 1023).astype(np.uint64)
    m = (_spread10(cell[:, 0]) << np.uint64(2)) | (_spread10(cell[:, 1]) << np.uint64(1)) | _spread10(cell[:, 2])
    b = 1
    while (1 << b) < n:
        b += 1
    return (m << np.uint64(b)) | np.arange(n, dtype=np.uint64), b


def lbvh(tri_enc: np.ndarray, leaf_n: int = 8, ploc_radius: int = 0):
    """(triangles in leaf order (n, 45), BVHNode_encoded nodes (m, 12)) as pt_bvh_build writes them; ploc_radius > 0
    rebuilds the tree above the LBVH leaves by PLOC (see ploc_top)."""
    t = np.asarray(tri_enc, np.float32).reshape(-1, 45)
    n = t.shape[0]
    k, b = keys(t)
    ks = np.sort(k)
    order = (ks & np.uint64((1 << b) - 1)).astype(np.int64)
    kl = [int(x) for x in ks]

    def clz(x: int) -> int:
        return 64 - x.bit_length()

    # radix tree: child[i] = (left, right) element refs; element e < n - 1 internal, n - 1 + p primitive p
    child = {}
    rng = {}
    parent = np.full(2 * n - 1, -1, np.int64)
    stack = [(0, n - 1, 0)] if n > 1 else []
    while stack:
        f, l, idx = stack.pop()
        common = clz(kl[f] ^ kl[l])
        lo_, hi_ = f, l - 1  # last s in [f, l-1] with clz(k[f]^k[s]) > common
        while lo_ < hi_:
            mid = (lo_ + hi_ + 1) // 2
            if clz(kl[f] ^ kl[mid]) > common:
                lo_ = mid
            else:
                hi_ = mid - 1
        g = lo_
        le = (n - 1 + g) if f == g else g
        re = (n - 1 + g + 1) if g + 1 == l else g + 1
        child[idx] = (le, re)
        rng[idx] = (f, l)
        parent[le] = idx
        parent[re] = idx
        if f != g:
            stack.append((f, g, g))
        if g + 1 != l:
            stack.append((g + 1, l, g + 1))

    # boxes, bottom-up with the kernel's operand order
    so = t[order]
    plo = _gmin(so[:, 0:3], _gmin(so[:, 3:6], so[:, 6:9]))
    phi = _gmax(so[:, 0:3], _gmax(so[:, 3:6], so[:, 6:9]))
    box_lo = np.zeros((2 * n - 1, 3), np.float32)
    box_hi = np.zeros((2 * n - 1, 3), np.float32)
    box_lo[n - 1:] = plo
    box_hi[n - 1:] = phi
    for i in sorted(child, key=lambda i: rng[i][1] - rng[i][0]):  # children before parents (smaller ranges first)
        a, c = child[i]
        box_lo[i] = _gmin(box_lo[a], box_lo[c])
        box_hi[i] = _gmax(box_hi[a], box_hi[c])

    def size(e):
        return rng[e][1] - rng[e][0] + 1 if e < n - 1 else 1

    keep = np.array([1 if parent[e] < 0 else int(size(parent[e]) > leaf_n) for e in range(2 * n - 1)], np.int64)
    if ploc_radius > 0 and n > 1:
        leaves = []  # reachable LBVH leaves: (first, count, lo, hi), in Morton (first) order
        for e in np.nonzero(keep)[0]:
            if e >= n - 1 or size(e) <= leaf_n:
                f0 = rng[e][0] if e < n - 1 else e - (n - 1)
                leaves.append((f0, size(e), box_lo[e], box_hi[e]))
        leaves.sort(key=lambda q: q[0])
        return np.ascontiguousarray(so), ploc_top(leaves, ploc_radius)
    ids = np.concatenate([[0], np.cumsum(keep)[:-1]])
    nodes = np.zeros((1 + int(keep.sum()), 12), np.float32)
    nodes[0] = DUMMY_NODE
    for e in np.nonzero(keep)[0]:
        o = nodes[1 + ids[e]]
        if e < n - 1 and size(e) > leaf_n:
            a, c = child[e]
            o[0], o[1] = 1 + ids[a], 1 + ids[c]
        else:
            o[3] = size(e)
            o[4] = rng[e][0] if e < n - 1 else e - (n - 1)
        o[6:9] = box_lo[e]
        o[9:12] = box_hi[e]
    return np.ascontiguousarray(so), nodes


def ploc_top(leaves, r: int) -> np.ndarray:
    """BVHNode_encoded nodes of the tree PLOC (Meister & Bittner 2018) builds over the given leaves, as the kernels
    ploc_nn / ploc_flags / ploc_compact / ploc_emit do: each cluster picks, among the clusters within r positions,
    the one whose merged box has the least half area ((dx*dy + dy*dz) + dz*dx in float32; ties: the sibling i ^ 1
    first, then the smaller pair),
    mutual pairs merge into a new node at the lower position (children in position order), the array is compacted.
    Node ids: PLOC node k (creation order) -> 1 + (M - 2 - k), leaf L -> M + L; node 0 the dummy."""
    M = len(leaves)
    C = np.array([~L for L in range(M)], np.int64)
    cl = np.array([q[2] for q in leaves], np.float32).reshape(M, 3)
    ch = np.array([q[3] for q in leaves], np.float32).reshape(M, 3)
    kids, klo, khi = [], [], []
    n = M
    while n > 1:
        idx = np.arange(n)
        best = np.full(n, np.inf, np.float32)
        bs = np.ones(n, np.int64)
        bj = np.full(n, -1, np.int64)
        # pairs ranked by (area, j != i ^ 1, min(i, j), max(i, j)) (kernels_bvh.hip ploc_nn)
        for off in range(-r, r + 1):  # ascending j: the first minimum wins
            if off == 0:
                continue
            j = idx + off
            valid = (j >= 0) & (j < n)
            jj = np.clip(j, 0, n - 1)
            with np.errstate(invalid="ignore"):  # union in position order (lower position first)
                if off < 0:
                    d = _gmax(ch[jj], ch) - _gmin(cl[jj], cl)
                else:
                    d = _gmax(ch, ch[jj]) - _gmin(cl, cl[jj])
                a = (d[:, 0] * d[:, 1] + d[:, 1] * d[:, 2]) + d[:, 2] * d[:, 0]
            a = np.where(np.isnan(a), np.float32(np.inf), a)  # NaN boxes rank last
            sj = (j != (idx ^ 1)).astype(np.int64)
            better = valid & ((bj < 0) | (a < best) | ((a == best) & (sj < bs)))
            best = np.where(better, a, best)
            bs = np.where(better, sj, bs)
            bj = np.where(better, j, bj)
        bj = np.where(bj < 0, idx, bj)
        mutual = (bj != idx) & (bj[bj] == idx)
        newf = mutual & (idx < bj)
        keepf = ~(mutual & (idx > bj))
        pos = np.cumsum(keepf) - keepf
        k0 = len(kids)
        knew = k0 + np.cumsum(newf) - newf
        C2 = np.empty(int(keepf.sum()), np.int64)
        cl2 = np.empty((len(C2), 3), np.float32)
        ch2 = np.empty((len(C2), 3), np.float32)
        for i in np.nonzero(keepf)[0]:
            p = pos[i]
            if newf[i]:
                j = bj[i]
                lo, hi = _gmin(cl[i], cl[j]), _gmax(ch[i], ch[j])
                k = int(knew[i])
                while len(kids) <= k:
                    kids.append(None)
                    klo.append(None)
                    khi.append(None)
                kids[k], klo[k], khi[k] = (int(C[i]), int(C[j])), lo, hi
                C2[p], cl2[p], ch2[p] = k, lo, hi
            else:
                C2[p], cl2[p], ch2[p] = C[i], cl[i], ch[i]
        C, cl, ch, n = C2, cl2, ch2, len(C2)

    def nid(ref):
        return 1 + (M - 2 - ref) if ref >= 0 else M + ~ref

    nodes = np.zeros((2 * M, 12), np.float32)
    nodes[0] = DUMMY_NODE
    for k, (a, b) in enumerate(kids):
        o = nodes[nid(k)]
        o[0], o[1] = nid(a), nid(b)
        o[6:9], o[9:12] = klo[k], khi[k]
    for L, (f0, cnt, lo, hi) in enumerate(leaves):
        o = nodes[M + L]
        o[3], o[4] = cnt, f0
        o[6:9], o[9:12] = lo, hi
    return nodes


def check_tree(tri_sorted: np.ndarray, nodes: np.ndarray, leaf_n: int) -> dict:
    """Structural validity of BVHNode_encoded nodes over triangles in leaf order: a binary tree reachable from node 1,
    every triangle in exactly one leaf, leaves of 1..leaf_n triangles, every box the exact glm min/max of the
    triangles below it. Returns {leaves, depth}; raises AssertionError otherwise."""
    t = np.asarray(tri_sorted, np.float32).reshape(-1, 45)
    n = t.shape[0]
    tlo = _gmin(t[:, 0:3], _gmin(t[:, 3:6], t[:, 6:9]))
    thi = _gmax(t[:, 0:3], _gmax(t[:, 3:6], t[:, 6:9]))
    seen = np.zeros(n, np.int64)
    visited = np.zeros(len(nodes), bool)
    leaves, depth = 0, 0
    stack = [(1, 1)]
    while stack:
        i, d = stack.pop()
        assert 1 <= i < len(nodes) and not visited[i], f"node {i} unreachable, repeated or out of range"
        visited[i] = True
        depth = max(depth, d)
        f = nodes[i]
        cnt, first = int(f[3]), int(f[4])
        if cnt > 0:
            assert cnt <= leaf_n and 0 <= first and first + cnt <= n, f"leaf {i}: ({cnt}, {first})"
            seen[first:first + cnt] += 1
            leaves += 1
            lo, hi = tlo[first:first + cnt].min(0), thi[first:first + cnt].max(0)
            if not np.isfinite(t[first:first + cnt, :9]).all():
                lo = hi = None  # NaN vertices: the box depends on the union order (glm min/max), not checked
        else:
            a, c = int(f[0]), int(f[1])
            stack += [(a, d + 1), (c, d + 1)]
            lo = hi = None
        if lo is not None:
            assert np.array_equal(f[6:9], lo, equal_nan=True) and np.array_equal(f[9:12], hi, equal_nan=True), \
                f"leaf {i} box"
    assert visited[1:].all(), "nodes not reachable from the root"
    assert (seen == 1).all(), "a triangle is in no leaf or in several"
    # interior boxes: the union of their children's boxes
    for i in range(1, len(nodes)):
        f = nodes[i]
        if int(f[3]) == 0:
            a, c = nodes[int(f[0])], nodes[int(f[1])]
            if np.isfinite(f[6:12]).all() and np.isfinite(a[6:12]).all() and np.isfinite(c[6:12]).all():
                assert np.array_equal(f[6:9], np.minimum(a[6:9], c[6:9])), f"node {i} AA"
                assert np.array_equal(f[9:12], np.maximum(a[9:12], c[9:12])), f"node {i} BB"
    return {"leaves": leaves, "depth": depth}
