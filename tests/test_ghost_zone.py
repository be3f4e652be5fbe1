"""The ghost zone's margins (ptsvgf.dist.svgf_margins, FrameShardRenderer): each SVGF pass draws its band widened by
its margin, and only the histories cross ranks. Checked on the CPU oracle over synthetic planes on which every pixel
is a surface pixel with a young history — so every tap of every pass is taken (7x7 variance, 25 a-trous taps, the
reprojection's bilinear taps and TAA's neighbourhood) and the widest reach of each stencil is exercised.

Everything a band does not hold is poison: NaN in the G-buffer, history and intermediate planes (NaN survives the
edge-stopping weights, even a zero-weight tap's 0 * NaN), arbitrary finite values in the path tracer's planes (the
reprojection zeroes a NaN illumination, svgf_reproject.frag:95-96). The band's rows must equal the whole-frame chain
bit for bit — and shrinking any one margin, or the history exchange, by a single row must change them."""
import numpy as np
import pytest

import oracle_ref as O
from ptsvgf.dist import REPROJ_REACH, motion_rows, svgf_margins

W, H = 24, 280
Y0, Y1 = 130, 150
ITERS = 5


def _inputs(seed, max_motion_rows):
    rng = np.random.default_rng(seed)

    def plane(lo, hi):
        return rng.uniform(lo, hi, (H, W, 4)).astype(np.float32)

    # one smooth surface (normals within a few degrees, depth within a fraction of its fwidth): the edge-stopping
    # weights (svgf_Atrous.frag:43-55) stay well above 0 for every tap, so every tap carries its input
    n = np.array([0.0, 0.0, 1.0]) + rng.normal(scale=0.02, size=(H, W, 3))
    n /= np.linalg.norm(n, axis=-1, keepdims=True)
    z = 0.5 + rng.uniform(-1e-4, 1e-4, (H, W, 1))
    nd = np.concatenate([n, z], -1).astype(np.float32)  # linear z != 1: surface
    fw = plane(0.001, 0.02)
    fw[..., 2] = nd[..., 3]
    vel = np.zeros((H, W, 4), np.float32)
    vel[..., 0] = rng.uniform(-2.0, 2.0, (H, W)) / W
    vel[..., 1] = rng.choice([-max_motion_rows, max_motion_rows], (H, W)) / H  # the largest motion, both ways
    vel[..., 3] = 1.0
    pm = plane(0.0, 1.0)
    pm[..., 2] = 1.0  # history length 1 -> 2: young (7x7 variance), and a valid reprojection blends half history
    prev_nd = nd + rng.normal(scale=1e-3, size=nd.shape).astype(np.float32)  # reprojection valid almost everywhere
    prev_nd[..., 3] = nd[..., 3]
    return dict(nd=nd, fwidth=fw, velocity=vel, prev_nd=prev_nd, color=plane(0.0, 2.0), albedo=plane(0.1, 1.0),
                emission=plane(0.0, 0.2), prev_illum=plane(0.0, 1.0), prev_moments=pm, prev_taa=plane(0.0, 1.0))


def _chain(inp, rows, taa=True, frame_counter=3):
    """reproject -> variance -> a-trous x ITERS -> modulate -> TAA; rows(stage) = rows a stage's output is right on
    (everything else poisoned with NaN), or None for the whole frame."""
    def cut(a, stage):
        r = rows(stage)
        if r is None:
            return a
        a = a.copy()
        a[:r[0]] = np.nan
        a[r[1]:] = np.nan
        return a

    ri, rm = O.reproject(inp["velocity"], inp["color"], inp["albedo"], inp["emission"], inp["prev_illum"],
                         inp["prev_moments"], inp["nd"], inp["prev_nd"], inp["fwidth"], np.float32(1.0 / W),
                         np.float32(1.0 / H), 10.0, 16.0, 2)
    ri, rm = cut(ri, "reproject"), cut(rm, "reproject")
    a = cut(O.variance(ri, rm, inp["nd"], inp["fwidth"], 4.0, 128.0, 2), "variance")
    for i in range(ITERS):
        a = cut(O.atrous(a, inp["nd"], inp["fwidth"], 1 << i, 4.0, 128.0, 2), "atrous")
    m = cut(O.modulate(inp["albedo"], inp["emission"], a, inp["nd"], 2), "modulate")
    if not taa:
        return dict(atrous=a, modulate=m)
    t = cut(O.taa(m, inp["prev_taa"], inp["velocity"], inp["nd"], frame_counter, 2), "taa")
    return dict(atrous=a, modulate=m, taa=t)


def _band_inputs(inp, margins, mrows, history_rows=None, zone=None, prev_nd_rows=None):
    """What a band holds: the G-buffer on the reprojection's rows + REPROJ_REACH (BandPlan.gbuffer_rows), the previous
    one on as many or, with the history exchange, margin + motion rows; the path tracer's planes on the reprojection's
    rows (finite garbage elsewhere); the histories on margin + motion rows (TAA: motion rows)."""
    rng = np.random.default_rng(99)
    out = dict(inp)
    g = margins["reproject"] + REPROJ_REACH  # BandPlan.gbuffer_rows
    nd_rows = max(g, margins["reproject"] + mrows) if prev_nd_rows is None else prev_nd_rows
    for k, rr in (("nd", g), ("fwidth", g), ("velocity", g), ("prev_nd", nd_rows)):
        a = inp[k].copy()
        lo, hi = max(0, Y0 - rr), min(H, Y1 + rr)
        if k == "prev_nd":  # NaN would pass the reprojection's validity tests (NaN > threshold is false): a
            a[:lo] *= np.float32([-1, -1, -1, 1.5])  # surface that fails them (svgf_reproject.frag:26-40)
            a[hi:] *= np.float32([-1, -1, -1, 1.5])
        else:
            a[:lo] = np.nan
            a[hi:] = np.nan
        out[k] = a
    z = margins["reproject"] if zone is None else zone
    for k in ("color", "albedo", "emission"):  # garbage of the same distribution (edge-stopping weights stay > 0)
        a = inp[k].copy()
        a[:Y0 - z] = rng.permutation(a[:Y0 - z].reshape(-1)).reshape(a[:Y0 - z].shape)
        a[Y1 + z:] = rng.permutation(a[Y1 + z:].reshape(-1)).reshape(a[Y1 + z:].shape)
        out[k] = a
    n = margins["reproject"] + mrows if history_rows is None else history_rows
    for k, rr in (("prev_illum", n), ("prev_moments", n), ("prev_taa", mrows)):
        a = inp[k].copy()
        a[:Y0 - rr] = np.nan
        a[Y1 + rr:] = np.nan
        out[k] = a
    return out


def _rows_of(margins):
    return lambda stage: (max(0, Y0 - margins[stage]), min(H, Y1 + margins[stage]))


@pytest.fixture(scope="module")
def case():
    mmax = 9.6  # rows of |motion.y|
    inp = _inputs(7, mmax)
    mrows = motion_rows(float(np.abs(inp["velocity"][..., 1]).max()), H)
    assert mrows == 10 + REPROJ_REACH
    return inp, mrows, {taa: _chain(inp, lambda s: None, taa) for taa in (False, True)}


@pytest.mark.parametrize("taa", [False, True])
def test_ghost_zone_band_equals_whole_frame(case, taa):
    inp, mrows, full = case
    margins = svgf_margins(ITERS, taa=taa)
    assert margins == {"taa": 0, "modulate": 2 * taa, "atrous": 60 + 2 * taa, "variance": 62 + 2 * taa,
                       "reproject": 65 + 2 * taa}
    got = _chain(_band_inputs(inp, margins, mrows), _rows_of(margins), taa)
    for k in got:
        a, b = got[k][Y0:Y1], full[taa][k][Y0:Y1]
        assert not np.isnan(a).any(), k
        assert np.array_equal(a.view(np.uint32), b.view(np.uint32)), k


@pytest.mark.parametrize("what,taa", [("reproject", False), ("variance", False), ("atrous", False), ("zone", False),
                                      ("history", False), ("prev_nd", False), ("taa_history", True)])
def test_ghost_zone_each_margin_is_needed(case, what, taa):
    """One row less anywhere and the band's rows change (or turn NaN). The path tracer's outermost zone row reaches
    the band only through the variance channel of the a-trous output (svgf_Atrous.frag:109-118), which modulate
    drops: the a-trous plane is part of the band's output (bench band_parity compares it). With TAA every margin
    carries 2 more rows for TAA's 3x3 neighbourhood (dist.TAA_NEIGHBOURS: +-1 texel and the GL LINEAR fetch's
    zero-weight row; kernels_taa.hip reads texels, +-1), so that extra row is not tight and is not tested here."""
    inp, mrows, full = case
    margins = svgf_margins(ITERS, taa=taa)
    m = dict(margins)
    zone, hist, taa_rows, nd_rows = None, None, mrows, None
    if what in m:
        m[what] -= 1
    elif what == "zone":
        zone = margins["reproject"] - 1
    elif what == "history":  # REPROJ_REACH is the taps' reach with rounding slack: cut into the motion itself
        hist = margins["reproject"] + mrows - REPROJ_REACH - 1
    elif what == "prev_nd":  # the previous normal/depth exchanged with the history, one row short of the motion
        nd_rows = margins["reproject"] + mrows - REPROJ_REACH - 1
    else:
        taa_rows = mrows - REPROJ_REACH - 1
    band = _band_inputs(inp, margins, taa_rows, history_rows=hist if hist is not None else margins["reproject"] + mrows,
                        zone=zone, prev_nd_rows=nd_rows)
    got = _chain(band, _rows_of(m), taa)
    same = [np.array_equal(np.nan_to_num(got[k][Y0:Y1], nan=-1.0).view(np.uint32), full[taa][k][Y0:Y1].view(np.uint32))
            for k in got]
    assert not all(same), what


@pytest.mark.parametrize("iters", range(0, 9))
@pytest.mark.parametrize("taa", [False, True])
def test_margins_keep_early_history_safe(iters, taa):
    """the early history exchange overwrites the iteration-1 output's and the normal/depth rows outside the
    band while iterations 2.. still run; svgf_margins asserts that nothing the band's rows depend on reads a row whose
    local bits can differ from the owner's (dist._check_early_history). A margin cut by one row must trip it."""
    from ptsvgf.dist import ATROUS_HALO, _check_early_history

    m = svgf_margins(iters, taa)  # does not raise
    if iters >= 2:
        bad = dict(m, variance=m["variance"] - 1)
        with pytest.raises(AssertionError):
            _check_early_history(bad, iters)
        # reading normal/depth beyond the G-buffer's rows
        bad = dict(m, reproject=sum(ATROUS_HALO[:iters]) - REPROJ_REACH - 1)
        with pytest.raises(AssertionError):
            _check_early_history(bad, iters)


def test_ghost_zone_band_needs_pt_source():
    """a ghost-zone band draws SVGF margin rows that its own path tracer never draws; without a pt_source
    providing them (FrameShardRenderer) BandRenderer refuses instead of silently differing from a frame."""
    from ptsvgf.dist import BandRenderer

    with pytest.raises(ValueError, match="pt_source"):
        BandRenderer(None, 64, 64, None, 0, 2, None, ghost_zone=True)
