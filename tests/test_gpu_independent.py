"""The GPU's full-size bench frame against the independent float64 restatement of path_tracing.frag (VERDICT r05 weak
1: the full-size 1080p / 4K checks compare the HIP path with the oracle only, and both share glsl_builtins.h).

tests/test_independent_pt.py's Restatement (numpy float64 from the shader's text, numpy's own transcendentals,
brute-force closest hits, nothing from glsl_builtins.h) traces 32 x 32 crops of the 4K bench frame the GPU rendered
(aspect-corrected primary rays, the full 2048 x 1024 environment): on the default camera the crops holding the most
wood (clearcoat), brass (metallic) and leaf (sheen) pixels, and on the surface-dominated camera the most leafy crop at
frameCounter 3. Same bar as the oracle's, over the union of a frame's crops: per channel within 1e-3 relative on all but
1 % of the pixels (branch flips between float64 and fp32 decisions), colour median relative difference at fp32 rounding
(path_tracing.frag:1056-1128). The restatement takes from GL that float(uint) rounds to fp32, that sampler weights are
8-bit fixed point, and that the varying pix arrives in fp32."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

MATERIALS = {"wood": (0.45, 0.28, 0.14), "brass": (0.80, 0.62, 0.35), "leaf": (0.16, 0.42, 0.12)}
CROP = 32
W, H = 3840, 2160


def _best_crop(albedo, colour):
    """The CROP x CROP window (on a CROP grid) holding the most pixels of this base colour."""
    m = np.all(np.abs(albedo[..., :3] - np.asarray(colour, np.float32)) < 1e-3, -1)
    g = m[:H - H % CROP, :W - W % CROP].reshape(H // CROP, CROP, W // CROP, CROP).sum((1, 3))
    j, i = np.unravel_index(int(np.argmax(g)), g.shape)
    return (int(i) * CROP, int(j) * CROP, CROP, CROP), int(g[j, i])


# bench.py's VIEWS (orbit radius, elevation, azimuth, look-at: Utils/camera.h:14-38 parameters)
VIEWS = {"default": None, "surface": dict(r_dis=0.8, upAngle=70.0, rotatAngle=180.0, move_vec=(0.4, -0.25, 0.0))}


def _frame(gl, scene, view, frames):
    from ptsvgf.camera import parameter_config, rigid_inverse
    from ptsvgf.renderer import Renderer

    r = Renderer(scene, W, H, parameter_config(), mode="fast", aspect_corrected=True, run_taa=False, run_output=False)
    if VIEWS[view]:
        for k, v in VIEWS[view].items():
            setattr(r.camera, k, np.array(v, np.float32) if isinstance(v, tuple) else np.float32(v))
        r.camera.dirty = True
    for _ in range(frames):
        r.frame()
    cam = r.camera
    fc = int(cam.frameCounter) - 1
    eye, rot = cam.cam_position, rigid_inverse(cam.cam_view_mat)
    pl = r.planes()
    out = [gl.readback(pl[k]) for k in ("color", "emission", "albedo")]
    r.close()
    return out, fc, eye, rot


@pytest.mark.timeout(900)
@pytest.mark.parametrize("view,frames,materials", [("default", 1, ("wood", "brass", "leaf")),
                                                   ("surface", 4, ("leaf",))])
def test_gpu_4k_frame_matches_independent_restatement(gpu, scene_bench, view, frames, materials):
    from test_independent_pt import Restatement, _compare

    planes, fc, eye, rot = _frame(gpu, scene_bench, view, frames)
    rs = Restatement(scene_bench, cull_group=32)
    refs, mines = [[], [], []], [[], [], []]
    for name in materials:
        crop, n = _best_crop(planes[2], MATERIALS[name])
        assert n >= 64, (view, name, n)  # the crop really holds that material
        x0, y0, cw, ch = crop
        mine = rs.frame(W, H, fc, eye, rot, crop=crop, aspect=True)
        for j in range(3):
            refs[j].append(planes[j][y0:y0 + ch, x0:x0 + cw])
            mines[j].append(mine[j])
        f1, m1, l1 = _compare([p[y0:y0 + ch, x0:x0 + cw] for p in planes], mine)
        print(f"{view} fc {fc} {name} crop {crop} ({n} px): outside 1e-3 {f1:.4f}, median rel {m1:.2e}, "
              f"beyond 1e-5 {l1:.4f}")
    frac, med, loose = _compare([np.concatenate(a, 1) for a in refs], [np.concatenate(b, 1) for b in mines])
    lit = float(np.mean(np.concatenate(refs[0], 1)[..., :3] > 0))
    print(f"{view}: pixels outside 1e-3 {frac:.4f}, colour median relative difference {med:.2e}, beyond 1e-5 "
          f"{loose:.4f}, lit {lit:.2f}")
    assert lit > 0.5
    assert frac <= 0.01, frac  # branch flips + the brass's amplified rounding (measured on the CPU oracle: brass crop
    #                            1.4 %, leaf crop 0.3 %; the bar is on the union of the frame's crops)
    assert med <= 1e-6, med    # fp32 rounding
    # channels beyond 1e-5 relative: the brass's metallic GGX lobe (a sharp D term) amplifies fp32 rounding of N.H
    # (24-27 % of a brass crop's channels on the CPU oracle, 12 % of a leaf crop's)
    assert loose <= 0.2, loose


@pytest.mark.timeout(900)
def test_gpu_4k_svgf_matches_independent_restatement(gpu, scene_bench):
    """The GPU's production SVGF chain at 4K against tests/test_independent_svgf.py's float64 restatement of the
    shaders (numpy's pow / exp / sqrt, texture fetches written out; nothing from glsl_builtins.h): two static frames,
    then an orbited frame whose history is reprojected with real sub-texel motion. On three 48 x 48 crops holding
    surface pixels, within north_star's 1e-3 per-channel L-inf (relative above 1): the reprojection
    (svgf_reproject.frag:26-204) from the GPU's own previous-frame planes, its texture coordinates in fp32 as GLSL's
    vec2 computes them (in float64 a real motion's taps land on the other side of the sampler's 8-bit rounding steps
    on ~0.5 % of the pixels); and the chain from the GPU's reprojected planes — variance (svgf_variance.frag), a-trous
    iteration 1 (the next frame's history), all five a-trous iterations (svgf_Atrous.frag, 62 rows of margin) and
    modulate."""
    from ptsvgf.camera import parameter_config
    from ptsvgf.renderer import Renderer
    from test_independent_svgf import atrous_ref, modulate_ref, reproject_ref, variance_ref

    gl = gpu
    r = Renderer(scene_bench, W, H, parameter_config(), mode="fast", aspect_corrected=True, run_taa=False,
                 run_output=False)
    for _ in range(2):
        r.frame()
    pl = r.planes()
    prev = {k: gl.readback(pl[k]) for k in ("history_illum", "reproj_moments", "normal_depth")}
    r.camera.orbit(1.0, 0.5)
    r.frame()
    pl = r.planes()
    cur = {k: gl.readback(pl[k]) for k in ("velocity", "color", "albedo", "emission", "normal_depth", "fwidth",
                                           "reproj_illum", "reproj_moments", "variance", "history_illum", "atrous",
                                           "modulate")}
    r.close()
    surf = cur["normal_depth"][..., 3] != 1.0
    M, C = 70, 48
    # crops: the 48 x 48 windows (on a 48 grid, at least M from the frame edges) with the most surface pixels in three
    # bands of columns (left, middle, right thirds)
    g = surf[:H - H % C, :W - W % C].reshape(H // C, C, W // C, C).sum((1, 3))
    crops = []
    for third in range(3):
        lo, hi = third * (W // C) // 3, (third + 1) * (W // C) // 3
        best = None
        for j in range(2, H // C - 2):
            for i in range(max(lo, 2), min(hi, W // C - 2)):
                if best is None or g[j, i] > g[best]:
                    best = (j, i)
        crops.append((best[1] * C, best[0] * C))
    worst = {}

    def rel(got, want, inner=None):
        d = np.abs(got[..., :3].astype(np.float64) - want[..., :3]) / np.maximum(1.0, np.abs(want[..., :3]))
        return float(np.nanmax(d)), float(np.mean(d.max(-1) > 1e-3))

    for x0, y0 in crops:
        assert surf[y0:y0 + C, x0:x0 + C].sum() >= 256, (x0, y0)
        oi, om = reproject_ref(cur["velocity"], cur["color"], cur["albedo"], cur["emission"], prev["history_illum"],
                               prev["reproj_moments"], cur["normal_depth"], prev["normal_depth"], cur["fwidth"],
                               crop=(x0, y0, C, C), coords32=True)
        inner = (slice(y0, y0 + C), slice(x0, x0 + C))
        for name, got, want in (("reproj_illum", cur["reproj_illum"][inner], oi),
                                ("reproj_moments", cur["reproj_moments"][inner], om)):
            mx, frac = rel(got, want)
            worst[name] = max(worst.get(name, (0, 0)), (frac, mx))
            assert mx <= 1e-3, (name, x0, y0, mx, frac)
        sl = (slice(y0 - M, y0 + C + M), slice(x0 - M, x0 + C + M))
        nd, fw = cur["normal_depth"][sl], cur["fwidth"][sl]
        a = variance_ref(cur["reproj_illum"][sl], cur["reproj_moments"][sl], nd, fw)
        chain = {"variance": a}
        for i in range(5):
            a = atrous_ref(a, nd, fw, 1 << i)
            if i == 1:
                chain["history_illum"] = a
        chain["atrous"] = a
        chain["modulate"] = modulate_ref(cur["albedo"][sl], cur["emission"][sl], a, nd)
        cin = (slice(M, M + C), slice(M, M + C))
        for name, want in chain.items():
            mx, frac = rel(cur[name][inner], want[cin])
            worst[name] = max(worst.get(name, (0, 0)), (frac, mx))
            assert mx <= 1e-3, (name, x0, y0, mx)
        young = int(np.sum((cur["reproj_moments"][inner][..., 2] < 4) & surf[inner]))
        print(f"crop ({x0}, {y0}): {int(surf[inner].sum())} surface px, {young} young-history px")
    print("worst (fraction beyond 1e-3, max relative):", {k: (round(f, 4), float(f"{m:.2e}")) for k, (f, m) in worst.items()})
