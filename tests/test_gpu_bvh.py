"""GPU LBVH builder (pt_bvh_build, csrc/kernels_bvh.hip) — SURVEY.md §8(f)2, dynamic scenes.

* The built buffers equal the CPU restatement (oracle/lbvh_ref.py) bit for bit: triangles in leaf order and
  BVHNode_encoded nodes, on the full bench scene and tiny / degenerate inputs, for several leaf sizes, as a plain
  LBVH and with the PLOC-built top; the trees are valid (every triangle in one leaf, exact boxes).
* Rendering over the GPU-built buffers (fast driver, frames in flight, every default switch) is bit-exact against
  the oracle path tracer walking the same buffers, before and after a rebuild for moved geometry.
The tree itself is not the reference's (buildBVHwithSAH, Utils/BVH.h:42-173, is a host sort-and-sweep): parity
of the builder against the reference is unpinned; the reference's formats and the walk over them are."""
import dataclasses
import os
import sys

import numpy as np
import pytest

import oracle_ref as O

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
import lbvh_ref as L  # noqa: E402

pytestmark = pytest.mark.gpu


def _build(gl, tri, leaf_n, ploc=0):
    src = gl.texture_buffer(tri)
    to = gl.texture_buffer(np.zeros(3, np.float32))
    no = gl.texture_buffer(np.zeros(3, np.float32))
    nodes, ms = gl.bvh_build(src, to, no, leaf_n, ploc)
    out = gl.buffer_readback(to).reshape(-1, 45), gl.buffer_readback(no).reshape(-1, 12)
    for h in (src, to, no):
        gl.destroy_texture(h)
    assert out[1].shape[0] == nodes
    return out, ms


def _random_tris(n, seed=0, flat_axis=None):
    rng = np.random.default_rng(seed)
    t = np.zeros((n, 45), np.float32)
    t[:, :9] = rng.uniform(-1, 1, (n, 9)).astype(np.float32)
    if flat_axis is not None:
        t[:, flat_axis:9:3] = 0.5
    t[:, 42] = np.arange(n)
    return t


@pytest.mark.parametrize("leaf_n,ploc", [(1, 0), (8, 0), (15, 0), (8, 16), (15, 16), (3, 32)])
def test_gpu_lbvh_equals_oracle_bench_scene(gpu, scene_bench, leaf_n, ploc):
    """(3, 32) is Renderer.rebuild_bvh's default."""
    (tri, nodes), ms = _build(gpu, scene_bench.tri_enc, leaf_n, ploc)
    want_tri, want_nodes = L.lbvh(scene_bench.tri_enc, leaf_n, ploc)
    assert np.array_equal(tri.view(np.uint32), want_tri.view(np.uint32))
    assert np.array_equal(nodes.view(np.uint32), want_nodes.view(np.uint32))
    info = L.check_tree(tri, nodes, leaf_n)
    print(f"bench scene {scene_bench.ntris} tris leaf_n {leaf_n} ploc {ploc}: {len(nodes)} nodes, "
          f"{info['leaves']} leaves, depth {info['depth']}, build {ms:.3f} ms")


@pytest.mark.parametrize("ploc", [0, 1, 16])
@pytest.mark.parametrize("n", [1, 2, 3, 17, 1000, 70000])
@pytest.mark.parametrize("flat", [None, 2])
def test_gpu_lbvh_equals_oracle_synthetic(gpu, n, flat, ploc):
    t = _random_tris(n, seed=n + 7, flat_axis=flat)
    (tri, nodes), _ = _build(gpu, t, 4, ploc)
    want_tri, want_nodes = L.lbvh(t, 4, ploc)
    assert np.array_equal(tri.view(np.uint32), want_tri.view(np.uint32))
    assert np.array_equal(nodes.view(np.uint32), want_nodes.view(np.uint32))


@pytest.mark.parametrize("ploc", [0, 16])
def test_gpu_lbvh_nan_vertices_equal_oracle(gpu, ploc):
    """Garbage input (NaN vertex positions): the device tree still equals the restatement bit for bit (NaN centroids
    out of the bounds, Morton cell 0; PLOC ranks NaN boxes last and terminates)."""
    t = _random_tris(300, seed=9)
    t[[5, 77, 150], 0] = np.nan
    (tri, nodes), _ = _build(gpu, t, 4, ploc)
    want_tri, want_nodes = L.lbvh(t, 4, ploc)
    assert np.array_equal(tri.view(np.uint32), want_tri.view(np.uint32))
    assert np.array_equal(nodes.view(np.uint32), want_nodes.view(np.uint32))


def test_gpu_lbvh_is_deterministic(gpu, scene_cornell):
    a, _ = _build(gpu, scene_cornell.tri_enc, 8)
    b, _ = _build(gpu, scene_cornell.tri_enc, 8)
    assert all(np.array_equal(x.view(np.uint32), y.view(np.uint32)) for x, y in zip(a, b))


def test_gpu_lbvh_rejects_bad_arguments(gpu):
    from ptsvgf._lib import PtError
    src = gpu.texture_buffer(_random_tris(4))
    to = gpu.texture_buffer(np.zeros(3, np.float32))
    for args in ((src, src, to, 8), (src, to, to, 8), (src, to, src, 8)):
        with pytest.raises(PtError):
            gpu.bvh_build(args[0], args[1], args[2], args[3])
    with pytest.raises(PtError):
        gpu.bvh_build(src, to, gpu.texture_buffer(np.zeros(3, np.float32)), 8, -1)
    no = gpu.texture_buffer(np.zeros(3, np.float32))
    for leaf_n in (0, 16):
        with pytest.raises(PtError):
            gpu.bvh_build(src, to, no, leaf_n)
    bad = gpu.texture_buffer(np.zeros(12, np.float32))  # not whole 45-float records
    with pytest.raises(PtError):
        gpu.bvh_build(bad, to, no, 8)
    for h in (src, to, no, bad):
        gpu.destroy_texture(h)


def _moved(scene, dy):
    """The plant (objIndex 2) lifted by dy: Triangle_encoded positions and the raster vertex list."""
    tri = scene.tri_enc.copy()
    sel = tri[:, 42] == 2.0
    for v in range(3):
        tri[sel, 3 * v + 1] += np.float32(dy)
    return tri


def test_render_over_gpu_lbvh_matches_oracle(gpu, scene_small):
    """Fast driver, 2 frames in flight, default switches, over GPU-built buffers; then the plant moves and the BVH
    is rebuilt in place (same buffer handles): path tracer outputs bit-exact vs the oracle on the same buffers."""
    from ptsvgf.renderer import Renderer

    W, H = 96, 64
    r = Renderer(scene_small, W, H, mode="fast", frames_in_flight=2, run_taa=False, run_output=False)
    r.rebuild_bvh(leaf_n=8, ploc_radius=16)
    tri, nodes = L.lbvh(scene_small.tri_enc, 8, 16)
    for step, (t_enc, want_tri, want_nodes) in enumerate([(scene_small.tri_enc, tri, nodes),
                                                          (_moved(scene_small, 0.05),) + L.lbvh(
                                                              _moved(scene_small, 0.05), 8, 0)]):
        if step == 1:  # the plain LBVH this time
            r.rebuild_bvh(tri_enc=t_enc, leaf_n=8, ploc_radius=0)
        got_tri = gpu.buffer_readback(r.trianglesTextureBuffer).reshape(-1, 45)
        got_nodes = gpu.buffer_readback(r.nodesTextureBuffer).reshape(-1, 12)
        assert np.array_equal(got_tri.view(np.uint32), want_tri.view(np.uint32))
        assert np.array_equal(got_nodes.view(np.uint32), want_nodes.view(np.uint32))
        sc = dataclasses.replace(scene_small, tri_enc=want_tri, node_enc=want_nodes)
        ref = O.OracleFrameLoop(sc, W, H, run_taa=False)
        for _ in range(step):  # the oracle reaches the renderer's frame counter (static camera)
            ref.frame()
        r.frame()
        want = ref.frame()
        got = {k: gpu.readback(v) for k, v in r.planes().items()}
        for key in ("color", "emission", "albedo"):
            assert np.array_equal(got[key].view(np.uint32), want[key].view(np.uint32)), (step, key)
    r.close()


@pytest.mark.parametrize("gbuffer_mode", [1, 0])
def test_device_raster_bind_equals_host_bind(gpu, scene_small, gbuffer_mode):
    """pt_raster_pass_bind_device (the G-buffer's tree built by the GPU builder from a device vertex list, records
    decoded on the device) after a move of the whole scene: G-buffer planes bit-identical to a renderer bound on the
    host to the moved vertex list — tile-binned rasterisation (mode 1) and the ray cast walking the tree (mode 0)."""
    from ptsvgf.renderer import Renderer

    W, H = 160, 96
    raster = scene_small.raster.reshape(-1, 6).copy()
    raster[:, 1] += np.float32(0.03)  # every vertex position up by 0.03 (pos3 + nrm3 per vertex)
    tri = scene_small.tri_enc.copy()
    tri[:, [1, 4, 7]] += np.float32(0.03)
    planes = ("normal_depth", "velocity", "fwidth", "world")
    out = []
    for device in (False, True):
        sc = dataclasses.replace(scene_small, raster=raster.reshape(-1)) if not device else scene_small
        r = Renderer(sc, W, H, mode="fast", run_taa=False, run_output=False)
        if device:
            r.rebuild_bvh(tri_enc=tri, raster=raster, leaf_n=8, ploc_radius=16)
        for p in r.init_pass:
            p.set_uniform_int("gbuffer_mode", gbuffer_mode)
        r.frame()
        got = r.planes()
        out.append({k: gpu.readback(got[k]) for k in planes})
        r.close()
    for k in planes:
        assert np.array_equal(out[0][k].view(np.uint32), out[1][k].view(np.uint32)), k
    assert 0.05 < float(np.mean(out[0]["normal_depth"][..., 3] != 1.0)) < 0.95


def test_raster_pass_share_rules(gpu, scene_small):
    """pt_raster_pass_share: both passes must be rasterize passes, the source bound on its own; a sharing pass draws
    the source's triangles (same G-buffer bits), and fails loudly once the source is destroyed."""
    from ptsvgf._lib import PtError
    from ptsvgf.gl import Rasterize_RenderPass, RenderPass, getShaderProgram, getTextureRGB32F

    W, H = 64, 48
    prog = getShaderProgram("shaders/rasterize_frag.frag", "shaders/rasterize_vert.vert")
    passes, outs = [], []
    for _ in range(2):
        p = Rasterize_RenderPass(prog, W, H)
        tex = [getTextureRGB32F(W, H) for _ in range(4)]
        p.colorAttachments += tex
        passes.append(p)
        outs.append(tex)
    a, b = passes
    a.bindData(scene_small.raster)
    b.bindData(np.zeros(18, np.float32))  # one degenerate triangle: replaced by the share below
    other = RenderPass(getShaderProgram("shaders/svgf_modulate.frag", "shaders/vert.vert"), W, H)
    other.colorAttachments.append(getTextureRGB32F(W, H))
    other.bindData(False)
    with pytest.raises(PtError):
        b.share_vertices(other)
    b.share_vertices(a)
    with pytest.raises(PtError):
        a.share_vertices(b)  # b is not bound on its own
    from ptsvgf.camera import Camera, mat_mul
    cam = Camera(W, H)
    cam.update()
    for p in (a, b):
        p.set_uniform_mat4("view", cam.cam_view_mat)
        p.set_uniform_mat4("projection", cam.cam_proj_mat)
        p.set_uniform_mat4("pre_viewproj", mat_mul(cam.cam_proj_mat, cam.cam_view_mat))
        p.draw()
    for ta, tb in zip(outs[0], outs[1]):
        assert np.array_equal(gpu.readback(ta).view(np.uint32), gpu.readback(tb).view(np.uint32))
    a.destroy()
    with pytest.raises(PtError):
        b.draw()
    b.destroy()
    other.destroy()


@pytest.mark.parametrize("case", ["point", "nan_object"])
def test_gpu_ploc_degenerate_runs_converge(gpu, case):
    """Runs of clusters with equal merge areas: 20 000 triangles collapsed to one point (every union
    area 0), or a whole object of NaN vertices (every area inf) beside a normal one. Pairs rank by (area, j != i ^ 1,
    min, max), so the sibling pairs of such a run are all mutual and it halves per iteration: the build completes
    (no iteration cap) and equals the restatement bit for bit, at Renderer.rebuild_bvh's defaults (3, 32)."""
    t = _random_tris(20000, seed=3)
    if case == "point":
        t[:, :9] = np.tile(np.float32([0.25, -0.5, 0.75]), 3)
    else:
        t[:12000, :9] = np.nan
    (tri, nodes), ms = _build(gpu, t, 3, 32)
    want_tri, want_nodes = L.lbvh(t, 3, 32)
    assert np.array_equal(tri.view(np.uint32), want_tri.view(np.uint32))
    assert np.array_equal(nodes.view(np.uint32), want_nodes.view(np.uint32))
    print(f"{case}: {len(nodes)} nodes, build {ms:.3f} ms")
    assert ms < 50.0  # tens of PLOC iterations, not thousands
