"""A second, independent restatement of the SVGF passes, in numpy float64 straight from the shaders' text
(svgf_reproject.frag, svgf_variance.frag, svgf_Atrous.frag, svgf_modulate.frag, output_pass.frag), against the
CPU oracle (oracle/, C, fp32).

The oracle and the HIP kernels share glsl_builtins.h, so a wrong built-in there would pass every kernel-vs-oracle
parity test. This restatement shares nothing with them: numpy's pow / exp / sqrt in float64, the shaders' own
order of operations, texel-centre sampling written out as index arithmetic. Agreement is to fp32 rounding
(relative 2e-4: pow(., 128) amplifies the fp32 rounding of the normal dot product about 128-fold). CPU only."""
import numpy as np
import pytest

import oracle_ref as O

RTOL, ATOL = 2e-4, 1e-5
PHI_COLOR, PHI_NORMAL = 4.0, 128.0


def _lum(c):
    return 0.2125 * c[..., 0] + 0.7154 * c[..., 1] + 0.0721 * c[..., 2]  # luminance(), svgf_Atrous.frag:57-59


def _weight(zc, zp, phi_depth, nc, np_, phi_normal, lc, lp, phi_illum):
    """computeWeight (svgf_Atrous.frag:43-55 = svgf_variance.frag:23-35). max(NaN, 0) is taken as 0 (fmax), the
    choice the oracle documents for 0 / 0 luminance terms."""
    wn = np.clip(np.sum(nc * np_, -1), 0.0, 1.0) ** phi_normal
    with np.errstate(divide="ignore", invalid="ignore"):
        wz = np.where(phi_depth == 0, 0.0, np.abs(zc - zp) / phi_depth)
        wl = np.abs(lc - lp) / phi_illum
    return np.exp(0.0 - np.fmax(wl, 0.0) - np.fmax(wz, 0.0)) * wn


def _shift(a, dy, dx):
    """a[y + dy, x + dx] for every (y, x), and whether that texel is inside the frame (the shaders' `inside`)."""
    H, W = a.shape[:2]
    ys, xs = np.arange(H) + dy, np.arange(W) + dx
    vy, vx = (ys >= 0) & (ys < H), (xs >= 0) & (xs < W)
    out = a[np.clip(ys, 0, H - 1)][:, np.clip(xs, 0, W - 1)]
    return out, vy[:, None] & vx[None, :]


def atrous_ref(illum, nd, fw, step):
    """svgf_Atrous.frag:61-126. computeVarianceCenter samples the centre nine times (its `p` is unused), with weights
    summing to 1: the centre's variance."""
    illum, nd, fw = (a.astype(np.float64) for a in (illum, nd, fw))
    kw = (1.0, 2.0 / 3.0, 1.0 / 6.0)
    var = illum[..., 3]
    zc, nc = nd[..., 3], nd[..., :3]
    lc = _lum(illum)
    phi_l = PHI_COLOR * np.sqrt(np.maximum(0.0, 1e-10 + var))
    phi_d = np.maximum(fw[..., 1], 1e-8) * step
    sw = np.ones(illum.shape[:2])
    s = illum.copy()
    for yy in range(-2, 3):
        for xx in range(-2, 3):
            if xx == 0 and yy == 0:
                continue
            ip, inside = _shift(illum, yy * step, xx * step)
            ndp, _ = _shift(nd, yy * step, xx * step)
            w = _weight(zc, ndp[..., 3], phi_d * np.hypot(xx, yy), nc, ndp[..., :3], PHI_NORMAL, lc, _lum(ip),
                        phi_l) * (kw[abs(xx)] * kw[abs(yy)])
            w = np.where(inside, w, 0.0)
            sw += w
            s[..., :3] += w[..., None] * ip[..., :3]
            s[..., 3] += w * w * ip[..., 3]
    out = np.concatenate([s[..., :3] / sw[..., None], (s[..., 3] / (sw * sw))[..., None]], -1)
    return np.where((zc == 1.0)[..., None], illum, out)


def variance_ref(illum, moments, nd, fw):
    """svgf_variance.frag:39-117: history length < 4 -> the 7x7 cross-bilateral moments, else pass-through."""
    illum, moments, nd, fw = (a.astype(np.float64) for a in (illum, moments, nd, fw))
    h = moments[..., 2]
    zc, nc = nd[..., 3], nd[..., :3]
    lc = _lum(illum)
    phi_d = np.maximum(fw[..., 1], 1e-8) * 3.0
    sw = np.zeros(illum.shape[:2])
    si = np.zeros(illum.shape[:2] + (3,))
    sm = np.zeros(illum.shape[:2] + (2,))
    for yy in range(-3, 4):
        for xx in range(-3, 4):
            ip, inside = _shift(illum, yy, xx)
            mp, _ = _shift(moments, yy, xx)
            ndp, _ = _shift(nd, yy, xx)
            w = _weight(zc, ndp[..., 3], phi_d * np.hypot(xx, yy), nc, ndp[..., :3], PHI_NORMAL, lc, _lum(ip),
                        PHI_COLOR)
            w = np.where(inside, w, 0.0)
            sw += w
            si += ip[..., :3] * w[..., None]
            sm += mp[..., :2] * w[..., None]
    sw = np.maximum(sw, 1e-6)
    si /= sw[..., None]
    sm /= sw[..., None]
    with np.errstate(divide="ignore", invalid="ignore"):
        v = (sm[..., 1] - sm[..., 0] * sm[..., 0]) * (4.0 / h)
    young = np.concatenate([si, v[..., None]], -1)
    young = np.where((zc == 1.0)[..., None], illum, young)
    return np.where((h < 4.0)[..., None], young, illum)


def modulate_ref(albedo, emission, illum, nd):
    """svgf_modulate.frag:18-29."""
    c = illum[..., :3].astype(np.float64)
    out = np.where((nd[..., 3] == 1.0)[..., None], c, c * albedo[..., :3] + emission[..., :3])
    return np.concatenate([out, np.ones(out.shape[:2] + (1,))], -1)


def _planes(seed, W=40, H=28):
    rng = np.random.default_rng(seed)
    yy, xx = np.mgrid[0:H, 0:W].astype(np.float64)
    n = np.stack([0.3 * np.sin(0.2 * xx), 0.3 * np.cos(0.15 * yy), np.ones_like(xx)], -1)
    n += rng.normal(0.0, 0.05, n.shape)
    n /= np.linalg.norm(n, axis=-1, keepdims=True)
    nd = np.concatenate([n, (0.5 + 0.002 * xx + 0.003 * yy + rng.normal(0, 1e-3, (H, W)))[..., None]], -1)
    nd[rng.uniform(size=(H, W)) < 0.1] = (0.2, 0.3, 0.3, 1.0)  # background: zCenter == 1
    illum = rng.uniform(0.0, 2.0, (H, W, 4))
    illum[..., 3] = rng.uniform(0.0, 0.3, (H, W))
    illum[3:6, 4:9, 3] = -1.0  # phiIllumination == 0
    fw = np.zeros((H, W, 4))
    fw[..., 1] = rng.uniform(0.0, 0.01, (H, W))
    fw[10:12, :, 1] = 0.0  # zero depth fwidth (the 1e-8 floor)
    moments = np.stack([rng.uniform(0, 1, (H, W)), rng.uniform(0, 2, (H, W)),
                        rng.choice([1.0, 2.0, 3.0, 4.0, 7.0], (H, W)), np.zeros((H, W))], -1)
    albedo, emission = rng.uniform(0, 1, (H, W, 4)), rng.uniform(0, 0.2, (H, W, 4))
    return {k: v.astype(np.float32) for k, v in dict(nd=nd, illum=illum, fw=fw, moments=moments, albedo=albedo,
                                                      emission=emission).items()}


def _close(got, want):
    assert got.shape == want.shape
    assert np.array_equal(np.isnan(got), np.isnan(want))
    ok = np.isclose(got, want, rtol=RTOL, atol=ATOL) | np.isnan(want)
    assert ok.all(), f"max |diff| {np.nanmax(np.abs(got - want)):.3e} at {np.argwhere(~ok)[:3].tolist()}"


@pytest.mark.parametrize("step", [1, 2, 4, 8, 16])
def test_atrous_oracle_matches_shader_restatement(step):
    p = _planes(3)
    _close(O.atrous(p["illum"], p["nd"], p["fw"], step, PHI_COLOR, PHI_NORMAL), atrous_ref(p["illum"], p["nd"], p["fw"], step))


def test_variance_oracle_matches_shader_restatement():
    p = _planes(4)
    _close(O.variance(p["illum"], p["moments"], p["nd"], p["fw"], PHI_COLOR, PHI_NORMAL),
           variance_ref(p["illum"], p["moments"], p["nd"], p["fw"]))


def test_modulate_oracle_matches_shader_restatement():
    p = _planes(5)
    _close(O.modulate(p["albedo"], p["emission"], p["illum"], p["nd"]),
           modulate_ref(p["albedo"], p["emission"], p["illum"], p["nd"]))


def output_ref(color):
    """output_pass.frag:12-24: tonrMapping(c, 1.5), then pow(c, 1 / 2.2); alpha 1."""
    c = color[..., :3].astype(np.float64)
    lum = 0.3 * c[..., 0] + 0.6 * c[..., 1] + 0.1 * c[..., 2]
    c = c * 1.0 / (1.0 + lum / 1.5)[..., None]
    with np.errstate(invalid="ignore"):
        c = c ** (1.0 / 2.2)
    return np.concatenate([c, np.ones(c.shape[:2] + (1,))], -1)


def test_output_oracle_matches_shader_restatement():
    c = _planes(6)["illum"] * 3.0  # non-negative colours (pow of a negative base is undefined in GLSL)
    _close(O.output(c), output_ref(c))


def tex_linear(img, u, v):
    """texture2D(img, (u, v)) under GL_LINEAR + GL_CLAMP_TO_EDGE (getTextureRGB32F, help_func.h:22-32): texel (i, j)
    centred at ((i + 0.5) / W, (j + 0.5) / H), the two nearest texels per axis blended, indices clamped to the edge;
    sub-texel weights in 8-bit fixed point, rounded (the texture-unit precision GL leaves to the implementation,
    SURVEY.md §7 hard part 3). A fetch at a texel centre returns that texel."""
    H, W = img.shape[:2]
    if isinstance(u, np.float32):  # an fp32 coordinate (GLSL's vec2): its texel position in fp32 too
        f = np.float32
        qx = float(np.floor((u * f(W) - f(0.5)) * f(256.0) + f(0.5)))
        qy = float(np.floor((v * f(H) - f(0.5)) * f(256.0) + f(0.5)))
    else:
        qx = np.floor((u * W - 0.5) * 256.0 + 0.5)
        qy = np.floor((v * H - 0.5) * 256.0 + 0.5)
    x0, y0 = int(qx // 256), int(qy // 256)
    ax, ay = (qx - 256.0 * x0) / 256.0, (qy - 256.0 * y0) / 256.0
    xa, xb = min(max(x0, 0), W - 1), min(max(x0 + 1, 0), W - 1)
    ya, yb = min(max(y0, 0), H - 1), min(max(y0 + 1, 0), H - 1)
    top = img[ya, xa] * (1.0 - ax) + img[ya, xb] * ax
    bot = img[yb, xa] * (1.0 - ax) + img[yb, xb] * ax
    return top * (1.0 - ay) + bot * ay


def reproject_ref(motion, color, albedo, emission, prev_illum, prev_moments, nd, prev_nd, fw, depth_thr=10.0,
                  normal_thr=16.0, crop=None, coords32=False):
    """svgf_reproject.frag:26-204. Every history fetch (the four taps' previous normal / depth, illumination and
    moments, the 3x3 fallback, the history length at uv - motion) is a LINEAR texture fetch (tex_linear); the
    current-frame planes are read at the pixel's own centre (plain texels). crop = (x0, y0, cw, ch): only those
    pixels of the whole frame (outputs cw x ch). coords32: the texture coordinates (uv, uv - motion, the taps, the
    shader's "bilinear weights") in fp32 as GLSL's vec2 computes them (a frame's real motion puts taps on the
    sampler's 8-bit rounding steps, where float64 coordinates round the other way); the rest stays float64."""
    H, W = color.shape[:2]
    x0, y0, cw, ch = crop if crop is not None else (0, 0, W, H)
    if crop is not None:  # the current-frame planes are read at the crop's pixels only; the history at any uv
        sl = (slice(y0, y0 + ch), slice(x0, x0 + cw))
        motion, color, albedo, emission, nd, fw = (a[sl] for a in (motion, color, albedo, emission, nd, fw))
    f = lambda a: a.astype(np.float64)  # noqa: E731
    motion, color, albedo, emission, prev_illum, prev_moments, nd, prev_nd, fw = map(
        f, (motion, color, albedo, emission, prev_illum, prev_moments, nd, prev_nd, fw))
    iw, ih = 1.0 / W, 1.0 / H
    oi, om = np.zeros((ch, cw, 4)), np.zeros((ch, cw, 4))
    for y in range(ch):
        for x in range(cw):
            if coords32:
                f = np.float32
                uv = np.array([(f(2 * (x0 + x) + 1) / f(W) - f(1)) * f(0.5) + f(0.5),
                               (f(2 * (y0 + y) + 1) / f(H) - f(1)) * f(0.5) + f(0.5)], np.float32)
            else:
                uv = np.array([(x0 + x + 0.5) * iw, (y0 + y + 0.5) * ih])
            zc = nd[y, x, 3]
            if zc == 1.0:
                oi[y, x], om[y, x] = color[y, x], prev_moments[y0 + y, x0 + x]
                continue
            with np.errstate(divide="ignore", invalid="ignore"):
                ill = (color[y, x, :3] - emission[y, x, :3]) / np.maximum(albedo[y, x, :3], 0.001)
            if np.isnan(ill).any():
                ill = np.zeros(3)
            prev = uv - motion[y, x, :2].astype(np.float32) if coords32 else uv - motion[y, x, :2]
            fwn, fwz = fw[y, x, 0], fw[y, x, 1]
            ncur = nd[y, x, :3]

            def valid_at(loc):
                if loc[0] < 0.0 or loc[0] > 1.0 or loc[1] < 0.0 or loc[1] > 1.0:
                    return False
                pnd = tex_linear(prev_nd, *loc)
                if abs(pnd[3] - zc) / (fwz + 1e-2) > depth_thr:
                    return False
                return not (np.linalg.norm(ncur - pnd[:3]) / (fwn + 1e-2) > normal_thr)

            offs = [(0.0, 0.0), (iw, 0.0), (0.0, ih), (iw, ih)]
            if coords32:
                iw32, ih32 = np.float32(1.0) / np.float32(W), np.float32(1.0) / np.float32(H)
                offs = [(0.0, 0.0), (iw32, 0.0), (0.0, ih32), (iw32, ih32)]
            v = [valid_at(prev + np.array(o, prev.dtype)) for o in offs]
            pi, pm, ok = np.zeros(4), np.zeros(2), any(v)
            if ok:
                if coords32:
                    f, iw32, ih32 = np.float32, np.float32(1.0) / np.float32(W), np.float32(1.0) / np.float32(H)
                    fx = float(prev[0] - f(int(prev[0] / iw32)) * iw32)
                    fy = float(prev[1] - f(int(prev[1] / ih32)) * ih32)
                else:
                    fx = prev[0] - int(prev[0] / iw) * iw  # the shader's "bilinear weights" in UV units (:84-91)
                    fy = prev[1] - int(prev[1] / ih) * ih
                wts = [(1 - fx) * (1 - fy), fx * (1 - fy), (1 - fx) * fy, fx * fy]
                sw = 0.0
                for k, o in enumerate(offs):
                    if v[k]:
                        loc = prev + np.array(o, prev.dtype)
                        pi += wts[k] * tex_linear(prev_illum, *loc)
                        pm += wts[k] * tex_linear(prev_moments, *loc)[:2]
                        sw += wts[k]
                ok = sw >= 0.01
                pi, pm = (pi / sw, pm / sw) if ok else (np.zeros(4), np.zeros(2))
            if not ok:
                n = 0.0
                for yy in (-1, 0, 1):
                    for xx in (-1, 0, 1):
                        loc = (prev + np.array([xx, yy], np.float32) * np.array(
                            [np.float32(1.0) / np.float32(W), np.float32(1.0) / np.float32(H)], np.float32)
                            if coords32 else prev + np.array([xx * iw, yy * ih]))
                        if valid_at(loc):
                            pi += tex_linear(prev_illum, *loc)
                            pm += tex_linear(prev_moments, *loc)[:2]
                            n += 1.0
                if n > 0:
                    ok = True
                    pi, pm = pi / n, pm / n
            if ok:
                hl = tex_linear(prev_moments, *prev)[2]
            else:
                pi, pm, hl = np.zeros(4), np.zeros(2), 0.0
            hl = min(32.0, hl + 1.0 if ok else 1.0)
            a = max(0.2, 1.0 / hl) if ok else 1.0
            m1 = _lum(ill)
            mom = (1.0 - a) * pm + a * np.array([m1, m1 * m1])
            oi[y, x, :3] = (1.0 - a) * pi[:3] + a * ill
            oi[y, x, 3] = max(0.0, mom[1] - mom[0] * mom[0])
            om[y, x, :2], om[y, x, 2] = mom, hl
    return oi, om


@pytest.mark.parametrize("subtexel", [False, True])
def test_reproject_oracle_matches_shader_restatement(subtexel):
    """Whole-texel motions (every tap on a texel centre) and sub-texel motions (the bilinear fetches the camera
    actually produces, svgf_reproject.frag:63-109 and :146). A sub-texel motion is (k + f) texels with f a multiple
    of 1/256 other than 1/2: every tap then sits on a step of the sampler's 8-bit sub-texel grid, half a step from
    where its rounding changes (and never on a texel boundary the shader's int() or the frame test could decide
    either way), so float64 and fp32 take the same sampler weights and the comparison tests the arithmetic, not a
    coin flip at a quantisation boundary. Invalid history (flipped normals, depth jumps), a fallback-only corner, a
    NaN sample."""
    H, W = 20, 24
    rng = np.random.default_rng(8 + int(subtexel))
    p = _planes(9, W, H)
    n = np.zeros((H, W, 3))
    n[..., 2] = 1.0
    n[..., :2] = rng.normal(0.0, 0.01, (H, W, 2))
    n /= np.linalg.norm(n, axis=-1, keepdims=True)
    nd = np.concatenate([n, np.full((H, W, 1), 0.5)], -1)
    nd[rng.uniform(size=(H, W)) < 0.08] = (0.2, 0.3, 0.3, 1.0)
    prev_nd = nd + np.concatenate([rng.normal(0, 0.005, (H, W, 3)), rng.normal(0, 1e-4, (H, W, 1))], -1)
    bad = rng.uniform(size=(H, W)) < 0.3  # clearly invalid history texels: flipped normals or a depth jump
    prev_nd[bad & (rng.uniform(size=(H, W)) < 0.5), :3] *= -1.0
    prev_nd[bad, 3] += np.where(rng.uniform(size=bad.sum()) < 0.5, 1.0, 0.0)
    prev_nd[:6, :6] *= (-1.0, -1.0, -1.0, 1.0)  # a corner where only the 3x3 fallback, or nothing, is valid
    fw = np.zeros((H, W, 4))
    fw[..., 0], fw[..., 1] = 0.05, 0.001
    yy, xx = np.mgrid[0:H, 0:W]
    mx = np.clip(rng.integers(-2, 3, (H, W)), xx - (W - 1), xx)  # uv - motion stays on a texel of the frame
    my = np.clip(rng.integers(-2, 3, (H, W)), yy - (H - 1), yy)
    if subtexel:
        fx, fy = rng.integers(1, 256, (H, W)), rng.integers(1, 256, (H, W))
        fx[fx == 128], fy[fy == 128] = 64, 192
        mx = mx + fx / 256.0 * rng.choice([-1.0, 1.0], (H, W))
        my = my + fy / 256.0 * rng.choice([-1.0, 1.0], (H, W))
    motion = np.zeros((H, W, 4))
    motion[..., 0], motion[..., 1] = mx / W, my / H
    color = p["illum"].astype(np.float64) * 2.0
    color[2, 3, :3] = np.nan  # a NaN path-tracer sample: illumination 0 (svgf_reproject.frag:176-178)
    moments = p["moments"].astype(np.float64)
    ins = [a.astype(np.float32) for a in (motion, color, p["albedo"], p["emission"], p["illum"], moments, nd,
                                          prev_nd, fw)]
    gi, gm = O.reproject(*ins, np.float32(1.0 / W), np.float32(1.0 / H))
    wi, wm = reproject_ref(*ins)
    _close(gi, wi)
    _close(gm, wm)
