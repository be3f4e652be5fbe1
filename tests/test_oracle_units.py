"""The oracle's building blocks against independent hand-derived values.

Parity for the GLSL passes is unpinned (no reference outputs exist, SURVEY.md
§8(c)); these tests pin each restated GLSL helper to values derived here
independently (numpy float64, closed forms, the shader text's own constants).
"""
import ctypes as C

import numpy as np
import pytest

import oracle_ref as O


def _f(a):
    return O.f32(a)


def _math(fn, x, y=None):
    x = _f(x)
    inp = x if y is None else _f(np.concatenate([x, _f(y)]))
    out = np.zeros(x.size, np.float32)
    O.lib().orc_math(fn, O.fp(inp), x.size, O.fp(out))
    return out


def _ulps(a, b):
    a = a.astype(np.float64)
    b32 = b.astype(np.float32)
    ulp = np.spacing(np.abs(b32)).astype(np.float64)
    return np.abs(a - b) / np.maximum(ulp, np.finfo(np.float32).tiny)


def test_builtin_transcendentals_accuracy():
    rng = np.random.default_rng(0)
    x = rng.uniform(-7, 7, 20000).astype(np.float32)
    for fn, ref in ((0, np.sin), (1, np.cos)):
        got = _math(fn, x)
        err = np.abs(got.astype(np.float64) - ref(x.astype(np.float64)))
        assert err.max() < 4e-7, (fn, err.max())
    y = rng.uniform(-3, 3, 20000).astype(np.float32)
    got = _math(2, y, x)
    assert np.abs(got - np.arctan2(y.astype(np.float64), x.astype(np.float64))).max() < 8e-7
    a = rng.uniform(-1, 1, 20000).astype(np.float32)
    assert _ulps(_math(3, a), np.arcsin(a.astype(np.float64))).max() <= 4
    p = np.exp(rng.uniform(-30, 30, 20000)).astype(np.float32)
    assert np.abs(_math(4, p) - np.log(p.astype(np.float64))).max() < 4e-6
    e = rng.uniform(-80, 80, 20000).astype(np.float32)
    assert _ulps(_math(5, e), np.exp(e.astype(np.float64))).max() <= 4


def _wang(seed):  # path_tracing.frag:438-445, independently restated
    s = seed & 0xFFFFFFFF
    s = (s ^ 61) ^ (s >> 16)
    s = (s * 9) & 0xFFFFFFFF
    s = s ^ (s >> 4)
    s = (s * 0x27D4EB2D) & 0xFFFFFFFF
    return s ^ (s >> 15)


@pytest.mark.parametrize("seed", [1, 3, 1973, 26699 | 1, 0xFFFFFFFF, 123456789])
def test_wang_hash(seed):
    assert O.lib().orc_wang_hash(seed) == _wang(seed)


def test_sobol_known_values():
    L = O.lib()
    # dimension 0 is the van der Corput sequence: bit-reversed index / 2^32
    for i in range(1, 64):
        rev = int(f"{i:032b}"[::-1], 2)
        assert L.orc_sobol(0, i) == np.float32(np.float32(rev) * np.float32(2.0 ** -32))
    # dimension 1 direction numbers (path_tracing.frag:465): V[1][0]=2^31, V[1][1]=3*2^30
    assert L.orc_sobol(1, 1) == 0.5
    assert L.orc_sobol(1, 2) == 0.75
    assert L.orc_sobol(1, 3) == 0.25


def _aabb(S, d, lo, hi):
    return O.lib().orc_hit_aabb(O.fp(_f(S)), O.fp(_f(d)), O.fp(_f(lo)), O.fp(_f(hi)))


def test_hit_aabb_semantics():
    lo, hi = [-1, -1, -1], [1, 1, 1]
    assert _aabb([0, 0, -5], [0, 0, 1], lo, hi) == 4.0            # entry distance t0
    assert _aabb([0, 0, 0], [0, 0, 1], lo, hi) == 1.0             # origin inside -> exit t1
    assert _aabb([0, 3, -5], [0, 0, 1], lo, hi) == -1.0           # miss
    assert _aabb([0, 0, 5], [0, 0, 1], lo, hi) <= 0.0             # behind: caller treats d<=0 as miss


def _tri(S, d, p, n=None):
    n = n if n is not None else np.tile([0, 0, 1], 3)
    out = np.zeros(5, np.float32)
    hit = O.lib().orc_hit_triangle(O.fp(_f(S)), O.fp(_f(d)), O.fp(_f(p)), O.fp(_f(n)), O.fp(out))
    return hit, out


def test_hit_triangle_semantics():
    P = [-1, -1, 0, 1, -1, 0, 0, 1, 0]  # CCW seen from +z: geometric N = +z
    hit, o = _tri([0, 0, 5], [0, 0, -1], P)
    assert hit and o[0] == 5.0 and o[4] == 0.0 and o[3] > 0        # front hit, smooth normal +z
    hit, o = _tri([0, 0, -5], [0, 0, 1], P)
    assert hit and o[4] == 1.0 and o[3] < 0                        # from behind: isInside, normal flipped
    hit, _ = _tri([0, 0, 5], [1, 0, 0], P)
    assert not hit                                                 # parallel (|N.d| < 1e-5)
    hit, _ = _tri([0, 0, 0.0001], [0, 0, -1], P)
    assert not hit                                                 # t < 0.0005
    hit, _ = _tri([5, 5, 5], [0, 0, -1], P)
    assert not hit                                                 # outside the edges


def _brdf(V, N, L, m):
    out = np.zeros(3, np.float32)
    O.lib().orc_brdf_eval(O.fp(_f(V)), O.fp(_f(N)), O.fp(_f(L)), O.fp(_f(m)), O.fp(out))
    return out


def _pdf(V, N, L, m):
    return O.lib().orc_brdf_pdf(O.fp(_f(V)), O.fp(_f(N)), O.fp(_f(L)), O.fp(_f(m)))


MAT = [0.8, 0.5, 0.3, 0.0, 0.2, 0.5, 0.0, 0.4, 0.0, 0.2, 0.5, 0.3, 0.7, 1.0]  # baseColor, subsurface, ...


def _unit(v):
    v = np.asarray(v, np.float64)
    return (v / np.linalg.norm(v)).astype(np.float32)


def test_brdf_zero_below_horizon_and_reciprocal():
    N = [0, 0, 1]
    V, L = _unit([0.3, 0.1, 0.9]), _unit([-0.5, 0.2, 0.6])
    assert (_brdf(V, N, _unit([0.1, 0, -1]), MAT) == 0).all()       # NdotL < 0 -> 0 (:623)
    assert _pdf(V, N, _unit([0.1, 0, -1]), MAT) == 0.0
    np.testing.assert_allclose(_brdf(V, N, L, MAT), _brdf(L, N, V, MAT), rtol=1e-5)  # Disney is reciprocal


def test_brdf_lambert_limit():
    """metallic 0, specular 0, roughness 1, no clearcoat/sheen/subsurface at normal incidence:
    f = baseColor/pi * Fd with Fd = mix(1,Fd90,FL)*mix(1,Fd90,FV); at L=V=N: FL=FV=0 -> f = baseColor/pi."""
    m = [0.5, 0.25, 1.0, 0.0, 0.0, 0.0, 0.0, 1.0, 0.0, 0.0, 0.5, 0.0, 1.0, 1.0]
    N = [0, 0, 1]
    f = _brdf(N, N, N, m)
    # specular=0 keeps Fs = mix(0, 1, FH) with FH=SchlickFresnel(1)=0 -> no spec term
    np.testing.assert_allclose(f, np.float32([0.5, 0.25, 1.0]) / np.float32(3.1415926), rtol=1e-6)


def test_brdf_pdf_normalised():
    """BRDF_Pdf integrates to ~1 over the hemisphere (lobe mixture of normalised pdfs)."""
    rng = np.random.default_rng(1)
    n = 6000
    u1, u2 = rng.random(n), rng.random(n)
    z = u1                                           # uniform hemisphere sampling, pdf 1/(2pi)
    r = np.sqrt(1 - z * z)
    Ls = np.stack([r * np.cos(2 * np.pi * u2), r * np.sin(2 * np.pi * u2), z], 1).astype(np.float32)
    V = _unit([0.2, 0.1, 0.95])
    m = [0.7, 0.7, 0.7, 0.0, 0.0, 0.5, 0.0, 0.6, 0.0, 0.0, 0.5, 0.0, 1.0, 1.0]
    vals = np.array([_pdf(V, [0, 0, 1], L, m) for L in Ls])
    est = vals.mean() * 2 * np.pi
    assert 0.85 < est < 1.15, est


def test_taa_oracle_properties():
    """taa.frag:126-135 pass-through cases and the steady state of the history clip."""
    rng = np.random.default_rng(7)
    H, W = 12, 16
    cur = rng.uniform(0.0, 2.0, (H, W, 4)).astype(np.float32)
    prev = rng.uniform(0.0, 2.0, (H, W, 4)).astype(np.float32)
    vel = np.zeros((H, W, 4), np.float32)
    nd = np.full((H, W, 4), 0.5, np.float32)
    nd[:3, :, 3] = 1.0                                   # background rows (clear colour .w == 1)
    out0 = O.taa(cur, prev, vel, nd, 0)                  # frameCounter 0: current colour
    assert np.array_equal(out0[..., :3], cur[..., :3]) and (out0[..., 3] == 1).all()
    out1 = O.taa(cur, prev, vel, nd, 5)
    assert np.array_equal(out1[:3, :, :3], cur[:3, :, :3])  # background: current colour
    # static history equal to a constant current image: clip box collapses, result is that colour
    c = np.broadcast_to(np.float32([0.3, 0.6, 0.9, 1.0]), (H, W, 4)).copy()
    out2 = O.taa(c, c, vel, nd, 5)
    assert np.allclose(out2[3:, :, :3], c[3:, :, :3], rtol=1e-5)
    # blend factor 0.05 with zero velocity: the result sits between the clipped history and the current colour
    lo = np.minimum(cur, prev)[3:, :, :3] - 1e-3
    assert np.isfinite(out1).all() and (out1[3:, :, :3] >= lo.min()).all()


def _quad_scene(mat, obj_index, textures):
    """One camera-facing quad (z = 0, [-1, 1]^2, uv = xy in [0, 1]) with the given material and material_array."""
    from ptsvgf.scene import POINT_LIGHTS, Scene, SceneBuilder, env_map, hdr_cache, transform

    b = SceneBuilder()
    pos = np.array([[-1, -1, 0], [1, -1, 0], [1, 1, 0], [-1, 1, 0]], np.float32)
    uv = (pos[:, :2] + 1.0) * 0.5
    b.add_mesh(pos, np.array([[0, 1, 2], [0, 2, 3]], np.int32), mat, transform(), False, obj_index, uvs=uv)
    b.build(8)
    tri, node, raster = b.encode()
    hdr = env_map(64, 32)
    return Scene("quad", tri, node, raster, POINT_LIGHTS.copy(), hdr, hdr_cache(hdr), b.counts(), textures)


def _quad_albedo(scene, W=24, H=24):
    from ptsvgf.camera import Camera, rigid_inverse

    cam = Camera(W, H)
    cam.update()
    col, em, al = O.OracleScene(scene).path_trace(W, H, 0, cam.cam_position, rigid_inverse(cam.cam_view_mat),
                                                  max_depth=1, threads=4)
    return al


def test_texture_array_branch_known_answers():
    """hitArray's texture branch (path_tracing.frag:315-364): a negative baseColor reads layer objIndex*4 of the
    RGBA8 material_array as c / 255; a constant layer gives that colour (to 2 ulp) wherever the quad is hit, the
    layer index follows objIndex, and with no array bound the fetch reads 0."""
    from ptsvgf.scene import material

    tex = np.zeros((8, 16, 16, 4), np.uint8)
    tex[4, :, :, :3] = (51, 102, 204)  # objIndex 1 -> layer 4 (albedo)
    tex[0, :, :, :3] = (255, 0, 0)     # objIndex 0's albedo layer: must not be read
    neg = material(baseColor=(-1.0, -1.0, -1.0))
    al = _quad_albedo(_quad_scene(neg, 1, tex))
    hit = al[..., 3] == 1.0
    lit = np.any(al[..., :3] != 0.0, axis=-1)
    assert lit.sum() > 100
    want = np.array([51, 102, 204], np.float32) / np.float32(255.0)
    # bilinear mixing of four equal texels, c*(1-a) + c*a, is exact up to float32 rounding (2 ulp)
    assert np.allclose(al[lit][:, :3], want, rtol=3e-7, atol=0)
    al0 = _quad_albedo(_quad_scene(neg, 1, None))  # no array bound: the fetch reads 0
    assert not np.any(al0[..., :3] != 0.0) and hit.any()
    pos = material(baseColor=(0.25, 0.5, 0.75))    # non-negative: the texture is never read
    alp = _quad_albedo(_quad_scene(pos, 1, tex))
    assert np.allclose(alp[lit][:, :3], [0.25, 0.5, 0.75])


def test_texture_array_bilinear_and_subrect_quirk():
    """GL_LINEAR + CLAMP_TO_EDGE on the RGBA8 layer, sampled at the quad's smooth uv (uv = (x+1)/2, (y+1)/2): a
    red ramp image occupying only the left half of the layer (the reference uploads each image at the origin of
    a larger layer, help_func.h:12). Left of the quad's centre line every hit reads the image (green = 1/255,
    red non-decreasing along the row, within the ramp's range); right of it the fetch reads the unwritten zero
    texels in every channel."""
    from ptsvgf.scene import material

    S, W = 32, 40
    tex = np.zeros((4, S, S, 4), np.uint8)
    tex[0, :, :S // 2, 0] = np.arange(S // 2, dtype=np.uint8)[None, :] * 16   # red ramp, left half only
    tex[0, :, :S // 2, 1:3] = 1
    al = _quad_albedo(_quad_scene(material(baseColor=(-1.0, -1.0, -1.0)), 0, tex), W=W, H=W)
    quad = np.abs(al[..., 2] - 1.0 / 255.0) < 1e-7  # blue = 1/255 exactly only where the image is read
    rows = [y for y in range(W) if quad[y].sum() > 4]
    assert len(rows) > 10
    for y in rows:
        xs = np.nonzero(quad[y])[0]
        assert xs.max() < W // 2 + 1                       # the image ends at the quad's centre line (uv.x = 0.5)
        red = al[y, xs, 0]
        assert np.all(np.diff(red) >= 0) and red.max() <= 240 / 255.0 + 1e-6 and red.min() >= 0.0
        right = al[y, W // 2 + 2:, :3]
        assert not np.any(right != 0.0)                    # beyond the image: zero texels (or sky misses)
