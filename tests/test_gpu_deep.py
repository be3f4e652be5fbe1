"""Trees the round-1 build refused: the drop-in now accepts every BVH the reference can walk.

* A reference BVH deeper than the 32-entry LDS traversal stack (the reference walks with int stack[256],
  path_tracing.frag:378): a "chain" tree (147 interior levels) over the Cornell scene's triangles in a seeded
  random order, so every leaf box spans the scene and a walk pushes one entry per level. The wavefront
  kernels switch to their spill variant (stack entries past the LDS stack in a per-pixel column of HBM); the
  trace counters show rays really spilled, and every path-tracer plane is bit-exact against the oracle, which
  walks the same chain with the reference's 256-entry stack. The megakernel (A/B only) refuses such trees loudly.
* Geometry whose SAH builds degenerate (400 exactly coincident triangles: every cut costs the same, so a sweep
  peels one primitive per level). The reference builder's tree gets 123 levels deep (walked with the spill
  stack); the build-side trees (G-buffer tree, any-hit tree) switch to balanced halves before they outgrow the
  stack. The scene renders bit-exact against the oracle, exact-t ties re-walked on the reference tree.
"""
import dataclasses

import numpy as np
import pytest

import oracle_ref as O

pytestmark = pytest.mark.gpu


def chain_bvh(tri_enc: np.ndarray, per_leaf: int = 15) -> np.ndarray:
    """Reference-encoded BVH (BVHNode_encoded, 12 floats: left, right, 0, n, index, 0, AA, BB; node 0 a dummy,
    root 1) over the triangles in index order: leaves of `per_leaf` consecutive triangles, each interior node
    holding one leaf and the rest of the chain. Boxes are exact unions, as buildBVHwithSAH makes them."""
    n = tri_enc.shape[0]
    P = tri_enc[:, :9].reshape(n, 3, 3)
    leaves = [(i, min(per_leaf, n - i)) for i in range(0, n, per_leaf)]
    L = len(leaves)
    lo = np.array([P[i:i + c].reshape(-1, 3).min(0) for i, c in leaves], np.float32)
    hi = np.array([P[i:i + c].reshape(-1, 3).max(0) for i, c in leaves], np.float32)
    node = np.zeros((2 * L, 12), np.float32)
    for j, (i, c) in enumerate(leaves):          # leaf j = node L + j
        node[L + j, 3], node[L + j, 4] = c, i
        node[L + j, 6:9], node[L + j, 9:12] = lo[j], hi[j]
    for k in range(L - 1):                       # interior I_k = node 1 + k: leaf k and the rest of the chain
        node[1 + k, 0] = L + k
        node[1 + k, 1] = 2 + k if k < L - 2 else 2 * L - 1
        node[1 + k, 6:9], node[1 + k, 9:12] = lo[k:].min(0), hi[k:].max(0)
    return node


def _pt_planes(gl, r):
    return {k: gl.readback(r.planes()[k]) for k in ("color", "emission", "albedo")}


def _check_bits(got, want, tag):
    for k in got:
        assert np.array_equal(got[k].view(np.uint32), want[k].view(np.uint32)), (tag, k)


def test_deep_reference_bvh_matches_oracle(gpu, scene_cornell):
    from ptsvgf._lib import PtError
    from ptsvgf.renderer import Renderer

    gl = gpu
    tri = scene_cornell.tri_enc[np.random.default_rng(7).permutation(scene_cornell.ntris)]
    deep = dataclasses.replace(scene_cornell, name="cornell_chain", tri_enc=tri, node_enc=chain_bvh(tri))
    W, H = 64, 48
    ref = O.OracleFrameLoop(deep, W, H, run_taa=False)
    want = [ref.frame() for _ in range(3)]
    ref3 = want[2]
    # production switches (closest hits on the SAH tree over these leaves, exact ties re-walked on the chain), then
    # every walk on the chain itself (closest_tree = shadow_tree = 0): the spill path carries those
    for switches in ({}, {"closest_tree": 0, "shadow_tree": 0}):
        r = Renderer(deep, W, H, mode="fast", run_taa=False, run_output=False)
        for k, v in switches.items():
            r.pass_path_tracing.set_uniform_int(k, v)
        r.frame()
        _check_bits(_pt_planes(gl, r), {k: want[0][k] for k in ("color", "emission", "albedo")}, switches)
        st = r.trace_stats()  # frame 1, counters on
        _check_bits(_pt_planes(gl, r), {k: want[1][k] for k in ("color", "emission", "albedo")}, switches)
        print(switches, st)
        if switches:
            assert st["spills"] > 0, st  # rays went past the 32-entry LDS stack
        r.close()
    # the spill columns of a batch (global pids): 3 frames drawn as one batch, frames in flight
    rb = Renderer(deep, W, H, mode="fast", run_taa=False, run_output=False, frames_in_flight=3, trace_batch=3)
    for _ in range(3):
        rb.frame()
    rb.flush()
    _check_bits(_pt_planes(gl, rb), {k: ref3[k] for k in ("color", "emission", "albedo")}, "batch")
    rb.close()
    r = Renderer(deep, W, H, mode="fast", run_taa=False, run_output=False)
    r.pass_path_tracing.set_uniform_int("pt_kernel", 1)
    with pytest.raises(PtError, match="megakernel"):
        r.frame()
    r.close()


def test_degenerate_sah_builds_fit_the_stack(gpu):
    """400 exactly coincident triangles left of the clock: the reference tree is 123 levels deep, the G-buffer
    and any-hit trees build depth-capped, and the frames match the oracle bit for bit (G-buffer, path tracer)."""
    from ptsvgf.renderer import Renderer
    from ptsvgf.scene import POINT_LIGHTS, Scene, SceneBuilder, env_map, hdr_cache, material, transform

    import os
    gl = gpu
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    b = SceneBuilder()
    b.add_obj(os.path.join(repo, "assets", "models", "clock.obj"), material(baseColor=(0.8, 0.6, 0.3)), transform(),
              True, 0)
    n = 400
    tri = np.array([[-1.0, -0.4, 1.2], [-0.2, -0.4, 1.2], [-0.6, 0.3, 1.2]], np.float32)  # left of the clock, nearer
    b.add_mesh(np.tile(tri, (n, 1)), np.arange(3 * n, dtype=np.int32).reshape(n, 3),
               material(baseColor=(0.3, 0.6, 0.8)), transform(), False, 1)
    b.build(8)
    t, nd, raster = b.encode()
    hdr = env_map(128, 64)
    scene = Scene("coincident", t, nd, raster, POINT_LIGHTS.copy(), hdr, hdr_cache(hdr), b.counts())
    print(scene.counts)
    assert scene.counts["max_depth"] > 64  # the reference builder chains the coincident triangles (123 levels)
    W, H = 64, 48
    ref = O.OracleFrameLoop(scene, W, H, run_taa=False)
    r = Renderer(scene, W, H, mode="fast", atrous_exact=True, run_taa=False, run_output=False)
    coop = Renderer(scene, W, H, mode="fast", atrous_exact=True, run_taa=False, run_output=False)
    coop.pass_path_tracing.set_uniform_int("closest_budget", 8)  # the cooperative walk meets the ties too
    coop.pass_path_tracing.set_uniform_int("trace_refill", 75)
    for f in range(2):
        r.frame()
        coop.frame()
        want = ref.frame()
        got = {k: gl.readback(v) for k, v in r.planes().items()}
        for k in ("normal_depth", "velocity", "fwidth", "world", "color", "emission", "albedo"):
            assert np.array_equal(got[k].view(np.uint32), want[k].view(np.uint32)), (f, k)
        gc = {k: gl.readback(coop.planes()[k]) for k in ("color", "emission", "albedo")}
        for k in gc:
            assert np.array_equal(gc[k].view(np.uint32), want[k].view(np.uint32)), ("coop", f, k)
        assert float(np.mean(want["albedo"][..., 2] > 0.7)) > 0.05  # the stacked triangles are in view
    st_coop = coop.trace_stats()
    print("cooperative", st_coop)
    assert st_coop["tie_rewalks"] > 0
    coop.close()
    st = r.trace_stats()
    print(st)
    assert st["tie_rewalks"] > 0  # coincident triangles meet the same t: re-walked on the reference tree
    r.close()
