"""Tile-shard transfers (pt_tiles_count / pt_tiles_copy, kernels_shard.hip; dist.TileShardRenderer): a rank's path
tracer draws the 16 x 16 tiles t = k * stride + offset of the frame (tile_stride / tile_offset), and each band owner
needs every rank's pixels of its band's rows. The packed layout is restated here in numpy (per segment: each plane,
each row, the row's subset tiles in x order) and the library is checked against it: the pixel counts on the CPU, the
bytes moved on the GPU, and a frame's subsets exchanged through packed buffers against the one-GPU frame."""
import numpy as np
import pytest

from ptsvgf import _lib


def subset_index(W, stride, offset, y0, y1, tile_y0=0):
    """(row, column) of every packed pixel of one plane of a segment, in packed order."""
    ntx = W // 16
    ys, xs = [], []
    for y in range(y0, y1):
        ty = (y - tile_y0) // 16
        for tx in range(ntx):
            if (ty * ntx + tx) % stride == offset:
                ys += [y] * 16
                xs += list(range(16 * tx, 16 * tx + 16))
    return np.array(ys, np.int64), np.array(xs, np.int64)


CASES = [(320, 3, 0, 0, 256, 0), (320, 3, 2, 5, 250, 0), (3840, 8, 7, 300, 701, 0), (1920, 8, 3, 0, 1080, 0),
         (96, 5, 4, 17, 33, 16), (48, 4, 1, 0, 40, 0), (64, 1, 0, 3, 9, 0)]


@pytest.mark.parametrize("W,stride,offset,y0,y1,tile_y0", CASES)
def test_tiles_count_matches_layout(W, stride, offset, y0, y1, tile_y0):
    import ctypes as C

    n = C.c_int64()
    assert _lib.pt().pt_tiles_count(W, tile_y0, stride, offset, y0, y1, C.byref(n)) == 0
    assert n.value == subset_index(W, stride, offset, y0, y1, tile_y0)[0].size


def test_tiles_count_subsets_partition_the_rows():
    import ctypes as C

    n = C.c_int64()
    for W, stride, y0, y1 in ((320, 3, 7, 201), (3840, 8, 0, 2160), (112, 5, 16, 31)):
        tot = 0
        for off in range(stride):
            assert _lib.pt().pt_tiles_count(W, 0, stride, off, y0, y1, C.byref(n)) == 0
            tot += n.value
        assert tot == W * (y1 - y0)


def test_tiles_count_refuses_bad_arguments():
    import ctypes as C

    n = C.c_int64()
    L = _lib.pt()
    assert L.pt_tiles_count(100, 0, 3, 0, 0, 16, C.byref(n)) == -6  # width not a multiple of 16
    assert L.pt_tiles_count(96, 0, 3, 3, 0, 16, C.byref(n)) == -6   # offset outside [0, stride)
    assert L.pt_tiles_count(96, 8, 3, 0, 0, 16, C.byref(n)) == -6   # rows before the tile origin


@pytest.mark.gpu
@pytest.mark.parametrize("W,H,stride", [(320, 256, 3), (96, 80, 8), (3840, 2160, 8)])
def test_tiles_copy_layout_and_round_trip(gpu, W, H, stride):
    """pack: every segment's block equals the numpy layout (several segments, one launch, rows not aligned to tiles,
    one stored in band storage with row0 > 0); unpack of those blocks into zeroed planes writes exactly the subset
    pixels and leaves the others untouched."""
    import torch

    gl = gpu
    rng = np.random.default_rng(W + stride)
    planes = [rng.standard_normal((H, W, 4)).astype(np.float32) for _ in range(3)]
    dev = [torch.from_numpy(p).cuda() for p in planes]
    tex = [gl.wrap_device_texture(t.data_ptr(), W, H) for t in dev]
    segs = [(0, H, 0), (5, H - 3, stride - 1), (H // 3, H // 3 + 40, min(1, stride - 1))]
    sizes = [gl.tiles_count(W, stride, o, a, b) for a, b, o in segs]
    bufs = [torch.full((3 * n, 4), np.nan, dtype=torch.float32, device="cuda") for n in sizes]
    from ptsvgf._lib import check, pt

    check(pt().pt_set_stream(torch.cuda.current_stream().cuda_stream))
    gl.tiles_copy(tex, stride, [(a, b, o, buf.data_ptr()) for (a, b, o), buf in zip(segs, bufs)], unpack=False)
    torch.cuda.synchronize()
    for (a, b, o), buf, n in zip(segs, bufs, sizes):
        ys, xs = subset_index(W, stride, o, a, b)
        got = buf.cpu().numpy().reshape(3, n, 4)
        for j in range(3):
            assert np.array_equal(got[j], planes[j][ys, xs]), (a, b, o, j)
    # unpack into band storage holding rows [r0, r0 + rows): the segment (a, b, o) must lie inside
    a, b, o = segs[2]
    r0, rows = a - 2, b - a + 7
    band = [torch.zeros((rows, W, 4), dtype=torch.float32, device="cuda") for _ in range(3)]
    gl.set_band(W, H, a, b, r0, rows)
    try:
        btex = [gl.wrap_device_texture(t.data_ptr(), W, H) for t in band]
    finally:
        gl.set_band(W, H, 0, H, 0, H)
    gl.tiles_copy(btex, stride, [(a, b, o, bufs[2].data_ptr())], unpack=True)
    torch.cuda.synchronize()
    ys, xs = subset_index(W, stride, o, a, b)
    for j in range(3):
        want = np.zeros((rows, W, 4), np.float32)
        want[ys - r0, xs] = planes[j][ys, xs]
        assert np.array_equal(band[j].cpu().numpy(), want), j
    with pytest.raises(Exception):  # rows outside the band storage
        gl.tiles_copy(btex, stride, [(a - 3, b, o, bufs[2].data_ptr())], unpack=True)
    for t in tex + btex:
        gl.destroy_texture(t)


@pytest.mark.gpu
def test_tile_subsets_exchanged_compose_to_frame(gpu, scene_small):
    """The tile shard's data path on one GPU: N subset draws of one frame, each packed per band zone (the pack a rank
    does for its peers), unpacked into each band's planes (the receiving rank's unpack of all N subsets): every
    band's zone rows equal the one-GPU frame's bit for bit."""
    import torch

    from ptsvgf.renderer import Renderer
    from ptsvgf.camera import parameter_config

    gl = gpu
    W, H, N = 160, 96, 3
    from ptsvgf._lib import check, pt

    check(pt().pt_set_stream(torch.cuda.current_stream().cuda_stream))
    a = Renderer(scene_small, W, H, parameter_config(), mode="fast", run_taa=False, run_output=False)
    a.frame()
    want = [gl.readback(a.planes()[k]) for k in ("color", "emission", "albedo")]
    zones = [(0, 40), (20, 70), (55, 96)]  # overlapping, like ghost-zone bands
    buf = {}
    for r in range(N):
        b = Renderer(scene_small, W, H, parameter_config(), mode="fast", run_taa=False, run_output=False)
        b.pass_path_tracing.set_uniform_int("tile_stride", N)
        b.pass_path_tracing.set_uniform_int("tile_offset", r)
        b.frame()
        pl = b.planes()
        tex = [pl[k] for k in ("color", "emission", "albedo")]
        for k, (z0, z1) in enumerate(zones):
            n = gl.tiles_count(W, N, r, z0, z1)
            buf[r, k] = torch.empty((3 * n, 4), dtype=torch.float32, device="cuda")
        gl.tiles_copy(tex, N, [(z0, z1, r, buf[r, k].data_ptr()) for k, (z0, z1) in enumerate(zones)], unpack=False)
        torch.cuda.synchronize()
        b.close()
    for k, (z0, z1) in enumerate(zones):
        planes = [torch.zeros((H, W, 4), dtype=torch.float32, device="cuda") for _ in range(3)]
        tex = [gl.wrap_device_texture(t.data_ptr(), W, H) for t in planes]
        gl.tiles_copy(tex, N, [(z0, z1, r, buf[r, k].data_ptr()) for r in range(N)], unpack=True)
        torch.cuda.synchronize()
        for j in range(3):
            assert np.array_equal(planes[j].cpu().numpy()[z0:z1], want[j][z0:z1]), (k, j)
        for t in tex:
            gl.destroy_texture(t)
    a.close()


@pytest.mark.gpu
def test_batched_tile_subsets_equal_single_draws(gpu, scene_small):
    """pt_pass_draw_batch of several frames' draws of ONE tile subset (a tile-shard rank batching its frames, so each
    traversal launch carries several subsets' rays) writes what each frame's own subset draw writes, bit for bit; a
    batch mixing subsets is refused."""
    import torch

    from ptsvgf.camera import parameter_config
    from ptsvgf.renderer import Renderer
    from ptsvgf._lib import check, pt

    gl = gpu
    W, H, N, B = 160, 96, 3, 3
    check(pt().pt_set_stream(torch.cuda.current_stream().cuda_stream))
    outs = []
    for batch in (1, B):
        r = Renderer(scene_small, W, H, parameter_config(), mode="fast", run_taa=False, run_output=False,
                     frames_in_flight=B, trace_batch=batch)
        r._stream_to(torch.cuda.current_stream())
        r.pass_path_tracing.set_uniform_int("tile_stride", N)
        r.pass_path_tracing.set_uniform_int("tile_offset", 1)
        r.pass_path_tracing.set_uniform_int("trace_refill", 90)
        passes = []
        for s in range(B):
            r._use_slot(s)
            r._path_trace()
            passes.append(r.pt_pass)
            r.camera.frameCounter += 1
        if batch > 1:
            gl.draw_batch(passes)
            with pytest.raises(Exception):  # one subset per batch
                passes[1].set_uniform_int("tile_offset", 2)
                gl.draw_batch(passes)
        torch.cuda.synchronize()
        outs.append([[gl.readback(t) for t in r.pt_slots[s][1]] for s in range(B)])
        r.close()
    for s in range(B):
        for j in range(3):
            assert np.array_equal(outs[0][s][j], outs[1][s][j]), (s, j)
    assert np.any(outs[0][1][0])  # the subset drew something
