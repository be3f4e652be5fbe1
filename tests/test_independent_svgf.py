"""A second, independent restatement of the SVGF passes, in numpy float64 straight from the shaders' text
(svgf_Atrous.frag, svgf_variance.frag, svgf_modulate.frag, output_pass.frag), against the CPU oracle (oracle/, C, fp32).

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
