"""The tile-binned G-buffer rasteriser (gbuffer_mode 1, the default: kernels_pt.hip gbuffer_raster_kernel) against
the ray cast it replaces (gbuffer_mode 0, gbuffer_kernel): the same definition (closest front-facing Moller hit of
the pixel-centre ray, ties to the lower triangle index, DESIGN.md "G-buffer definition"), so every G-buffer plane —
and everything downstream — must be bit-identical. The ray cast itself is pinned to the oracle by
test_gpu_parity.py and test_gpu_fullsize.py (which now run the rasteriser)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

GBUF = ("world", "normal_depth", "velocity", "fwidth")
MOVES = [None, (1.0, 0.75), (-1.5, -1.0), (20.0, 10.0)]


def _render(gl, scene, W, H, mode, moves, caps=None, rows=None, keys=GBUF + ("color", "atrous")):
    from ptsvgf.renderer import Renderer

    r = Renderer(scene, W, H, mode="fast", aspect_corrected=W != H, run_taa=False, run_output=False,
                 gbuffer_rows=rows)
    for p in r.init_pass:
        p.set_uniform_int("gbuffer_mode", mode)
    out = []
    for f, mv in enumerate(moves):
        if mv:
            r.camera.orbit(*mv)
        for p in r.init_pass:  # per frame: a pair-list cap (0: the allocation's) that may force an overflow
            p.set_uniform_int("raster_pair_cap", caps[f] if caps else 0)
        r.frame()
        out.append({k: gl.readback(r.planes()[k]) for k in keys})
    r.close()
    return out


def _same(a, b, tag, rows=None):
    for f, (fa, fb) in enumerate(zip(a, b)):
        for k in fa:
            x, y = fa[k], fb[k]
            if rows is not None:
                x, y = x[rows[0]:rows[1]], y[rows[0]:rows[1]]
            bad = np.argwhere(np.any(x.view(np.uint32) != y.view(np.uint32), axis=-1))
            assert len(bad) == 0, (tag, f, k, len(bad), bad[:5].tolist())


@pytest.mark.parametrize("scene_name", ["scene_small", "scene_cornell", "scene_nan"])
def test_raster_equals_ray_cast(gpu, scene_name, request):
    scene = request.getfixturevalue(scene_name)
    W, H = 160, 96
    _same(_render(gpu, scene, W, H, 1, MOVES), _render(gpu, scene, W, H, 0, MOVES), scene_name)


def test_raster_equals_ray_cast_bench_scene_1080p(gpu, scene_bench):
    """The bench scene at configs[1] size: 30 k triangles (the plant's foliage binned densely, the table and floor
    binned by whole blocks), a moving camera including a large orbit step."""
    W, H = 1920, 1080
    want = _render(gpu, scene_bench, W, H, 0, MOVES)
    _same(_render(gpu, scene_bench, W, H, 1, MOVES), want, "bench1080")
    # frames 1 and 2 overflow: the ray cast's fallback grid (a few hundred blocks, kernels_pt.hip gbuffer_fix_blocks)
    # strides over all 8 160 tiles, writes the frame and clears the tile counts; frame 3 bins from zero again
    _same(_render(gpu, scene_bench, W, H, 1, MOVES, caps=[0, 8, 8, 0]), want, "bench1080/overflow")


def test_raster_band_rows_and_overflow_fallback(gpu, scene_small):
    """A band of G-buffer rows (the multi-GPU case: boxes clipped to the band, tiles counted from its first row),
    and a pair list too small for the frame on frames 1 and 2 (the rasteriser flags the overflow, the ray cast
    writes the frame and clears the tile counts the skipped scatter left, so frame 3 bins from zero again)."""
    W, H = 160, 96
    rows = (21, 70)
    keys = GBUF
    want = _render(gpu, scene_small, W, H, 0, MOVES, rows=rows, keys=keys)
    _same(_render(gpu, scene_small, W, H, 1, MOVES, rows=rows, keys=keys), want, "band", rows)
    _same(_render(gpu, scene_small, W, H, 1, MOVES, caps=[0, 8, 8, 0], keys=keys),
          _render(gpu, scene_small, W, H, 0, MOVES, keys=keys), "overflow")


def _pt(gl, scene, W, H, raster, moves, cap=0, tree=1):
    from ptsvgf.renderer import Renderer

    r = Renderer(scene, W, H, mode="fast", aspect_corrected=W != H, run_taa=False, run_output=False)
    r.pass_path_tracing.set_uniform_int("primary_raster", raster)
    r.pass_path_tracing.set_uniform_int("raster_pair_cap", cap)
    r.pass_path_tracing.set_uniform_int("closest_tree", tree)
    out = []
    for mv in moves:
        if mv:
            r.camera.orbit(*mv)
        r.frame()
        out.append({k: gl.readback(r.planes()[k]) for k in ("color", "emission", "albedo")})
    st = r.trace_stats()
    r.close()
    return out, st


@pytest.mark.parametrize("scene_name", ["scene_small", "scene_cornell", "scene_nan"])
def test_primary_raster_equals_walk(gpu, scene_name, request):
    """Primary rays by tile-binned reference leaves (wf_primary_raster, the default) give the per-pixel walk's bits
    (wf_primary), through camera moves. The pixels the rasteriser flags (ties, nothing below the G-buffer bound)
    go to the wave-cooperative walk (wf_primary_coop) with the SAH tree on, to wf_primary's fixup without it; with
    a pair list too small for the frame every pixel is walked instead."""
    scene = request.getfixturevalue(scene_name)
    W, H = 160, 96
    want, st0 = _pt(gpu, scene, W, H, 0, MOVES)
    got, st1 = _pt(gpu, scene, W, H, 1, MOVES)
    _same(got, want, scene_name)
    assert st1["primary_rays"] == st0["primary_rays"] == W * H, (st0, st1)
    print(scene_name, "flagged primary pixels:", st1["primary_retries"], "tie rewalks:", st1["tie_rewalks"])
    over, _ = _pt(gpu, scene, W, H, 1, MOVES, cap=4)
    _same(over, want, scene_name + "/overflow")
    no_tree, _ = _pt(gpu, scene, W, H, 1, MOVES, tree=0)
    _same(no_tree, want, scene_name + "/no-tree")


def test_primary_raster_equals_walk_bench_scene_1080p(gpu, scene_bench):
    W, H = 1920, 1080
    want, _ = _pt(gpu, scene_bench, W, H, 0, MOVES)
    got, st = _pt(gpu, scene_bench, W, H, 1, MOVES)
    print(st)
    _same(got, want, "bench1080")
    # every subset's pair list overflows: wf_primary walks all 8 160 tiles from its fix-up grid of a few hundred
    # blocks striding over them (kernels_wavefront.hip primary_fix_blocks)
    over, _ = _pt(gpu, scene_bench, W, H, 1, MOVES, cap=4)
    _same(over, want, "bench1080/overflow")


def test_trace_stats_buffer_length_is_respected(gpu, scene_small):
    """pt_pass_set_trace_stats_n writes no counter past the caller's count, and the first-published entry point
    (pt_pass_set_trace_stats) writes its 12 counters only (the buffer grew from 12 to 14 counters)."""
    import ctypes as C

    import torch

    from ptsvgf._lib import pt
    from ptsvgf.renderer import Renderer

    assert pt().pt_trace_stats_count() == len(Renderer.STAT_KEYS) == 14
    r = Renderer(scene_small, 64, 48, mode="fast", run_taa=False, run_output=False)
    sentinel = -12345
    try:
        for n, setter in ((12, "v1"), (5, "n"), (14, "n")):
            buf = torch.zeros(16, dtype=torch.int64, device="cuda")
            buf[n:] = sentinel
            torch.cuda.synchronize()
            h = r.pass_path_tracing._handle()
            if setter == "v1":
                assert pt().pt_pass_set_trace_stats(h, C.c_void_p(buf.data_ptr())) == 0
            else:
                assert pt().pt_pass_set_trace_stats_n(h, C.c_void_p(buf.data_ptr()), n) == 0
            r.frame()
            r.flush()
            torch.cuda.synchronize()
            assert pt().pt_pass_set_trace_stats_n(h, None, 0) == 0
            got = buf.cpu().tolist()
            assert got[0] == 64 * 48, (n, got)  # primary rays
            assert all(v == sentinel for v in got[n:]), (n, got)
    finally:
        r.close()
