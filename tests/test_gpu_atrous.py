"""Production a-trous kernels (kernels_atrous.hip) against the exact oracle on
synthetic planes with the special cases the shader's arithmetic has: background
pixels (z == 1), phiIllumination == 0 (variance <= -1e-10) next to neighbours of
exactly equal luminance, zero depth fwidth, NaN normals. Bar: north_star's 1e-3
per channel (relative above 1).

Interior vs border: a tile of the LDS kernel takes its unchecked (interior) path
only when its whole dilated footprint lies inside the frame, i.e. columns
[x0 - 2S, x0 + 64*NX + 2S) and rows [ybase - 2S, ybase + S*(TJ+1)] with TJ = 8.
At 320x200 every S = 16 tile is a border tile (ybase >= 32 and ybase + 144 < 200
cannot both hold), so the S = 16 interior path is exercised by the 416x320
planes (tiles with x0 = 128, ybase in [128, 175]); `_interior_tiles` counts the
interior tiles of each case and the test requires at least one for every step."""
import numpy as np
import pytest

import oracle_ref as O

pytestmark = pytest.mark.gpu

SIZES = [(320, 200), (416, 320)]


def _interior_tiles(W, H, S):
    """Tiles of atrous_tile_kernel<S> (kernels_atrous.hip) that take the unchecked path at W x H."""
    nx = 2 if S >= 16 else 1
    n = 0
    for x0 in range(0, W, 64 * nx):
        for g in range((H + S * 8 - 1) // (S * 8)):
            for b in range(S):
                yb = g * S * 8 + b
                if x0 - 2 * S >= 0 and x0 + 64 * nx - 1 + 2 * S < W and yb - 2 * S >= 0 and yb + S * 9 < H:
                    n += 1
    return n


def _planes(seed=11, W=320, H=200):
    rng = np.random.default_rng(seed)
    yy, xx = np.mgrid[0:H, 0:W].astype(np.float32)
    illum = np.empty((H, W, 4), np.float32)
    illum[..., :3] = rng.uniform(0.0, 3.0, (H, W, 3))
    illum[..., 3] = rng.uniform(0.0, 0.5, (H, W))
    illum[40:60, 100:140, 3] = -1.0                 # phiIllumination == 0 ...
    illum[40:60, 100:140, :3] = 0.5                 # ... with neighbours of equal luminance
    illum[45, 120, :3] = 0.75
    n = np.stack([0.2 * np.sin(xx * 0.05), 0.2 * np.cos(yy * 0.07), np.ones_like(xx)], -1)
    n += rng.normal(0.0, 0.02, n.shape)
    n /= np.linalg.norm(n, axis=-1, keepdims=True)
    nd = np.empty((H, W, 4), np.float32)
    nd[..., :3] = n
    nd[..., 3] = 2.0 + 0.01 * xx + 0.02 * yy + rng.normal(0.0, 0.01, (H, W))
    bg = rng.uniform(size=(H, W)) < 0.08
    nd[bg] = (0.2, 0.3, 0.3, 1.0)                   # clear colour: background sentinel
    nd[150:152, 30:34, :3] = np.nan                 # NaN normals (degenerate faces)
    fw = np.zeros((H, W, 4), np.float32)
    fw[..., 1] = rng.uniform(0.0, 0.05, (H, W))
    fw[80:90, :, 1] = 0.0
    return illum, nd, fw


def _run(gl, illum, nd, fw, step, variant, **uniforms):
    from ptsvgf.gl import GL_TEXTURE_2D, RenderPass, getShaderProgram, getTextureRGB32F
    H, W, _ = illum.shape
    ti, tn, tf, to = (getTextureRGB32F(W, H) for _ in range(4))
    gl.upload_rgba(ti, illum)
    gl.upload_rgba(tn, nd)
    gl.upload_rgba(tf, fw)
    p = RenderPass(getShaderProgram("shaders/svgf_Atrous.frag", "shaders/vert.vert"), W, H)
    p.colorAttachments.append(to)
    p.bindData(False)
    p.set_uniform_float("gPhiColor", 4.0)
    p.set_uniform_float("gPhiNormal", 128.0)
    p.set_uniform_int("gStepSize", step)
    p.set_uniform_int("atrous_variant", variant)
    for name, val in uniforms.items():
        p.set_uniform_int(name, val)
    p.set_texture_uniform(GL_TEXTURE_2D, ti, "gIllumination")
    p.set_texture_uniform(GL_TEXTURE_2D, tn, "gNormalAndLinearZ")
    p.set_texture_uniform(GL_TEXTURE_2D, tf, "gNormalDepthFwidth")
    p.draw()
    out = gl.readback(to)
    p.destroy()
    for t in (ti, tn, tf, to):
        gl.destroy_texture(t)
    return out


@pytest.mark.parametrize("size", SIZES)
@pytest.mark.parametrize("variant", [0, 1, 2])
@pytest.mark.parametrize("step", [1, 2, 4, 8, 16])
def test_atrous_kernel_vs_oracle(gpu, step, variant, size):
    W, H = size
    illum, nd, fw = _planes(W=W, H=H)
    want = O.atrous(illum, nd, fw, step)
    got = _run(gpu, illum, nd, fw, step, variant)
    assert np.array_equal(np.isnan(got), np.isnan(want)), \
        f"NaN pattern differs: gpu {int(np.isnan(got).sum())} oracle {int(np.isnan(want).sum())}"
    d = np.abs(got.astype(np.float64) - want) / np.maximum(1.0, np.abs(want))
    mx = float(np.nanmax(d))
    print(f"{W}x{H} step {step} variant {variant}: max rel diff {mx:.3e} "
          f"(interior tiles of the tile kernel: {_interior_tiles(W, H, step)})")
    assert mx <= 1e-3


def test_interior_tiles_cover_every_step():
    """The SIZES above reach the unchecked path of every step (CPU-side geometry check)."""
    for step in (1, 2, 4, 8, 16):
        assert max(_interior_tiles(W, H, step) for W, H in SIZES) > 0, step
    assert _interior_tiles(320, 200, 16) == 0 and _interior_tiles(416, 320, 16) > 0


@pytest.mark.parametrize("size", SIZES)
@pytest.mark.parametrize("step", [1, 2, 4, 8, 16])
def test_tile_kernel_equals_step_kernel(gpu, step, size):
    """The LDS-tiled kernel (variant 0, with and without the per-tile surface flags; its interior tiles run the taps
    as straight-line code, border tiles test each tap) performs the step kernel's (variant 2) arithmetic in the same
    tap order: identical bits, NaNs included."""
    illum, nd, fw = _planes(seed=5, W=size[0], H=size[1])
    b = _run(gpu, illum, nd, fw, step, 2)
    cases = [(0, {}), (0, dict(atrous_tile_flags=0))]
    for v, kw in cases:
        a = _run(gpu, illum, nd, fw, step, v, **kw)
        assert np.array_equal(a.view(np.uint32), b.view(np.uint32)), (v, kw)


def test_tile_kernel_aux_flag_on_rendered_planes(gpu, scene_small):
    """On real G-buffer planes the tile kernel reads the compact depth-fwidth plane, whose sign bit carries the
    zCenter == 1 flag: same bits as the step kernel reading the full texels, every step, 1080p-like aspect."""
    from ptsvgf.gl import GL_TEXTURE_2D, RenderPass, getShaderProgram, getTextureRGB32F
    from ptsvgf.camera import parameter_config
    from ptsvgf.renderer import Renderer

    Wr, Hr = 200, 120
    r = Renderer(scene_small, Wr, Hr, parameter_config(), mode="fast", aspect_corrected=True, run_taa=False,
                 run_output=False)
    for _ in range(2):
        r.frame()
    pl = r.planes()
    nd = gpu.readback(pl["normal_depth"])
    assert 0.05 < float(np.mean(nd[..., 3] == 1.0)) < 0.95  # both background and surface pixels present
    outs = {}
    for variant in (0, 2):
        for step in (1, 2, 4, 8, 16):
            to = getTextureRGB32F(Wr, Hr)
            p = RenderPass(getShaderProgram("shaders/svgf_Atrous.frag", "shaders/vert.vert"), Wr, Hr)
            p.colorAttachments.append(to)
            p.bindData(False)
            p.set_uniform_float("gPhiColor", 4.0)
            p.set_uniform_float("gPhiNormal", 128.0)
            p.set_uniform_int("gStepSize", step)
            p.set_uniform_int("atrous_variant", variant)
            p.set_texture_uniform(GL_TEXTURE_2D, pl["variance"], "gIllumination")
            p.set_texture_uniform(GL_TEXTURE_2D, pl["normal_depth"], "gNormalAndLinearZ")
            p.set_texture_uniform(GL_TEXTURE_2D, pl["fwidth"], "gNormalDepthFwidth")
            p.draw()
            outs[variant, step] = gpu.readback(to)
            p.destroy()
            gpu.destroy_texture(to)
    r.close()
    for step in (1, 2, 4, 8, 16):
        assert np.array_equal(outs[0, step].view(np.uint32), outs[2, step].view(np.uint32)), step
