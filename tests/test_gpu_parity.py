"""GPU parity: the HIP path (through the C ABI) against the CPU oracle on the
same seeded inputs. Bar (BASELINE.json north_star): per-channel L-inf <= 1e-3 in
fp32. The exact-form kernels are built to reproduce the oracle bit for bit, so
the tests also report (and for the path tracer require) bit-exact agreement.
"""
import numpy as np
import pytest

import oracle_ref as O

pytestmark = pytest.mark.gpu

TOL = 1e-3  # north_star: 1e-3 per-channel L-inf (fp32)


def _cmp(name, got, want, tol=TOL, rel=False):
    assert got.shape == want.shape, (name, got.shape, want.shape)
    assert np.isfinite(got).all() == np.isfinite(want).all(), f"{name}: non-finite mismatch"
    d = np.abs(got.astype(np.float64) - want.astype(np.float64))
    if rel:
        d = d / np.maximum(1.0, np.abs(want.astype(np.float64)))
    mx = float(np.nanmax(d)) if d.size else 0.0
    exact = float(np.mean(got == want))
    print(f"{name}: max|diff|={mx:.3e} bit-exact={exact * 100:.3f}%")
    assert mx <= tol, f"{name}: L-inf {mx} > {tol}"
    return exact


def _renderer(scene, W, H, **kw):
    from ptsvgf.renderer import Renderer

    return Renderer(scene, W, H, **kw)


def _readback(gl, r):
    return {k: gl.readback(v) for k, v in r.planes().items()}


@pytest.mark.parametrize("W,H", [(64, 64), (96, 64), (37, 23), (5, 3)])
def test_frames_match_oracle(gpu, scene_small, W, H):
    """3 frames, static camera: every pass output vs the oracle frame loop."""
    gl = gpu
    r = _renderer(scene_small, W, H, mode="reference", atrous_exact=True, run_taa=False, run_output=False)
    ref = O.OracleFrameLoop(scene_small, W, H)
    for f in range(3):
        r.frame()
        want = ref.frame()
        got = _readback(gl, r)
        for key in ("normal_depth", "velocity", "fwidth", "world"):
            _cmp(f"f{f}/{key}", got[key], want[key], tol=1e-5)
        for key in ("color", "emission", "albedo"):
            ex = _cmp(f"f{f}/{key}", got[key], want[key])
            assert ex == 1.0, f"path tracer output {key} is not bit-exact ({ex})"
        for key in ("reproj_illum", "reproj_moments", "variance", "atrous", "history_illum", "modulate"):
            _cmp(f"f{f}/{key}", got[key], want[key], rel=True)


@pytest.mark.parametrize("normal_map", [False, True])
def test_texture_array_path_matches_oracle(gpu, normal_map):
    """The material_array branch (path_tracing.frag:315-364): the clock samples albedo / metallic / roughness
    layers objIndex*4 + {0, 1, 3} (and the normal-map layer with use_normal_map), the table only its metallic
    layer; synthetic RGBA8 layers uploaded at the origin of larger layers (ptsvgf.scene.material_layers).
    Path-tracer outputs bit-exact against the oracle, both drivers."""
    from ptsvgf.camera import parameter_config
    from ptsvgf.scene import build_scene

    gl = gpu
    scene = build_scene("textured", hdr_size=(256, 128))
    cfg = parameter_config()
    cfg.use_normal_texture = normal_map
    W, H = 80, 64
    for mode in ("reference", "fast"):
        r = _renderer(scene, W, H, config=cfg, mode=mode, atrous_exact=True, run_taa=False, run_output=False)
        ref = O.OracleFrameLoop(scene, W, H, cfg)
        for f in range(2):
            r.frame()
            want = ref.frame()
            got = _readback(gl, r)
            for key in ("color", "emission", "albedo"):
                ex = _cmp(f"{mode}/f{f}/{key}", got[key], want[key])
                assert ex == 1.0, f"path tracer output {key} is not bit-exact ({ex})"
            _cmp(f"{mode}/f{f}/modulate", got["modulate"], want["modulate"], rel=True)
        al = got["albedo"]
        textured = np.any(al[..., :3] != 0, axis=-1) & (np.abs(al[..., 0] - al[..., 1]) > 1e-3)
        assert textured.sum() > 20  # the checker albedo of the clock is visible
        r.close()


def test_moving_camera_matches_oracle(gpu, scene_small):
    """Orbiting camera: reprojection with non-zero motion, frameCounter resets (camera.h:71)."""
    gl = gpu
    W = H = 64
    r = _renderer(scene_small, W, H, mode="reference", atrous_exact=True, run_taa=False, run_output=False)
    ref = O.OracleFrameLoop(scene_small, W, H)
    for f in range(4):
        if f:
            r.camera.orbit(2.0, 0.5)
            ref.camera.orbit(2.0, 0.5)
        r.frame()
        want = ref.frame()
        got = _readback(gl, r)
        assert np.abs(want["velocity"][..., :2][want["normal_depth"][..., 3] != 1.0]).max() > 0 or f == 0
        for key in ("velocity", "color", "reproj_illum", "reproj_moments", "variance", "atrous", "modulate"):
            _cmp(f"f{f}/{key}", got[key], want[key], rel=True)


def test_cornell_teapot_matches_oracle(gpu, scene_cornell):
    """configs[0] scene (Cornell-style box + teapot stand-in), axis-aligned geometry edge cases."""
    gl = gpu
    W = H = 64
    r = _renderer(scene_cornell, W, H, mode="reference", atrous_exact=True, run_taa=False, run_output=False)
    ref = O.OracleFrameLoop(scene_cornell, W, H)
    r.frame()
    want = ref.frame()
    got = _readback(gl, r)
    for key in ("normal_depth", "color", "albedo", "modulate"):
        _cmp(key, got[key], want[key], rel=True)


@pytest.mark.parametrize("K", [1, 4])
def test_config0_cornell_teapot_512_matches_oracle(gpu, K):
    """configs[0] at its stated size: the Cornell box + teapot stand-in at 512x512, 1 spp, depth 2, the path tracer
    alone (SVGF plays no part in its planes). Production fast driver (G-buffer-bounded primaries, SAH trees, lane
    refill with K = 4 frames in flight), then bench.py config0's unhinted _path_trace: color / emission / albedo
    bit-exact against the oracle path tracer (path_tracing.frag:1056-1128) on frames 0-3."""
    from ptsvgf.camera import Camera, parameter_config, rigid_inverse
    from ptsvgf.scene import build_scene

    gl = gpu
    W = H = 512
    scene = build_scene("cornell_teapot")
    cfg = parameter_config()
    r = _renderer(scene, W, H, config=cfg, mode="fast", run_taa=False, run_output=False, frames_in_flight=K)
    osc = O.OracleScene(scene)
    cam = Camera(W, H)

    def want():
        cam.update()
        out = osc.path_trace(W, H, cam.frameCounter, cam.cam_position, rigid_inverse(cam.cam_view_mat),
                             cfg.clamp_threshold, cfg.max_tracing_depth, aspect_corrected=False)
        cam.frameCounter += 1
        return dict(zip(("color", "emission", "albedo"), out))

    for f in range(3):
        r.frame()
        exp = want()
        got = _readback(gl, r)
        assert r.camera.frameCounter == cam.frameCounter
        for key in ("color", "emission", "albedo"):
            ex = _cmp(f"K{K}/f{f}/{key}", got[key], exp[key])
            assert ex == 1.0, f"path tracer output {key} is not bit-exact ({ex})"
        assert np.count_nonzero(got["albedo"][..., :3].any(axis=-1)) > W * H // 2  # the box fills the frame
    if K == 1:  # bench.py config0's timed call: the path tracer without the G-buffer hint
        r._path_trace()
        r.camera.frameCounter += 1
        exp = want()
        for key, plane in zip(("color", "emission", "albedo"), (r.curColor, r.Emission, r.Albedo)):
            ex = _cmp(f"unhinted/{key}", gl.readback(plane), exp[key])
            assert ex == 1.0, f"unhinted path tracer output {key} is not bit-exact ({ex})"
    r.close()


def test_nan_normals_match_oracle(gpu, scene_nan):
    """Degenerate faces -> NaN vertex normals: both sides propagate NaN identically."""
    gl = gpu
    W = H = 64
    r = _renderer(scene_nan, W, H, mode="reference", atrous_exact=True, run_taa=False, run_output=False)
    ref = O.OracleFrameLoop(scene_nan, W, H)
    for f in range(2):
        r.frame()
        want = ref.frame()
        got = _readback(gl, r)
        assert np.isnan(want["normal_depth"]).any(), "probe scene must produce NaN normals"
        for key in ("normal_depth", "color", "emission", "albedo", "reproj_illum", "variance", "atrous", "modulate"):
            _cmp(f"f{f}/{key}", got[key], want[key], rel=True)


def test_prune_is_result_preserving(gpu, scene_small):
    """Closest-hit box pruning (kernels_pt.hip) changes no pixel versus the reference's full traversal."""
    gl = gpu
    W = H = 64
    outs = []
    for prune in (True, False):
        r = _renderer(scene_small, W, H, mode="fast", prune=prune, run_taa=False, run_output=False)
        r.frame()
        outs.append(gl.readback(r.planes()["color"]))
    assert np.array_equal(outs[0], outs[1])


@pytest.mark.parametrize("scene_name", ["scene_small", "scene_cornell", "scene_nan"])
def test_bvh4_shadows_are_result_preserving(gpu, scene_name, request):
    """Shadow rays on the 4-wide BVH give the same verdicts as the binary walk (any-hit is order-free)."""
    gl = gpu
    scene = request.getfixturevalue(scene_name)
    W, H = 96, 64
    outs = []
    for wide in (1, 0):
        r = _renderer(scene, W, H, mode="fast", run_taa=False, run_output=False)
        r.pass_path_tracing.set_uniform_int("shadow_bvh4", wide)
        for _ in range(2):
            r.frame()
        outs.append({k: gl.readback(r.planes()[k]) for k in ("color", "emission", "albedo")})
    for k in outs[0]:
        assert np.array_equal(outs[0][k], outs[1][k], equal_nan=True), k


@pytest.mark.parametrize("scene_name", ["scene_small", "scene_cornell", "scene_nan"])
def test_closest_tree_is_result_preserving(gpu, scene_name, request):
    """Closest-hit rays on the SAH tree over the reference leaves (closest_tree=1, exact-t ties re-walked on the
    reference tree) give the reference-order walk's bits (closest_tree=0). The Cornell box's axis-aligned quads
    put many rays on shared diagonal edges, where two triangles meet the same t."""
    gl = gpu
    scene = request.getfixturevalue(scene_name)
    W, H = 96, 64
    outs = []
    for tree in (1, 0):
        r = _renderer(scene, W, H, mode="fast", run_taa=False, run_output=False)
        r.pass_path_tracing.set_uniform_int("closest_tree", tree)
        for _ in range(2):
            r.frame()
        outs.append({k: gl.readback(r.planes()[k]) for k in ("color", "emission", "albedo")})
        r.close()
    for k in outs[0]:
        assert np.array_equal(outs[0][k].view(np.uint32), outs[1][k].view(np.uint32)), k


@pytest.mark.parametrize("scene_name", ["scene_small", "scene_nan"])
def test_cooperative_shadow_walk_is_result_preserving(gpu, scene_name, request):
    """Shadow rays past the step budget are finished by the wave-cooperative walk (kernels_wavefront.hip
    wf_shadow_coop): budgets 4 (nearly every ray, including LDS-stack overflows), 16 and 128 give the serial walk's
    bits (budget 0), from the one-ray-per-lane kernel and from the lane-refill kernel (trace_refill 75)."""
    gl = gpu
    scene = request.getfixturevalue(scene_name)
    W, H = 96, 64
    outs = []
    for budget, refill in ((0, 0), (4, 0), (16, 0), (128, 0), (4, 75), (16, 75), (128, 75)):
        r = _renderer(scene, W, H, mode="fast", run_taa=False, run_output=False)
        r.pass_path_tracing.set_uniform_int("shadow_budget", budget)
        r.pass_path_tracing.set_uniform_int("trace_refill", refill)
        for _ in range(2):
            r.frame()
        outs.append({k: gl.readback(r.planes()[k]) for k in ("color", "emission", "albedo")})
        r.close()
    for o in outs[1:]:
        for k in o:
            assert np.array_equal(outs[0][k], o[k], equal_nan=True), k


@pytest.mark.parametrize("scene_name", ["scene_small", "scene_cornell", "scene_nan"])
def test_cooperative_closest_walk_is_result_preserving(gpu, scene_name, request):
    """Bounce rays past the visit budget are finished by the wave-cooperative closest-hit walk (kernels_wavefront.hip
    wf_closest_coop, from the lane-refill kernel): budgets 2 (nearly every ray), 16 and 64 give the serial walk's
    bits, ray counts and tie re-walks."""
    gl = gpu
    scene = request.getfixturevalue(scene_name)
    W, H = 96, 64
    outs = []
    for budget in (0, 2, 16, 64):
        r = _renderer(scene, W, H, mode="fast", run_taa=False, run_output=False)
        r.pass_path_tracing.set_uniform_int("closest_budget", budget)
        r.pass_path_tracing.set_uniform_int("trace_refill", 75)
        for _ in range(2):
            r.frame()
        outs.append({k: gl.readback(r.planes()[k]) for k in ("color", "emission", "albedo")})
        r.close()
    for o in outs[1:]:
        for k in o:
            assert np.array_equal(outs[0][k].view(np.uint32), o[k].view(np.uint32)), k


@pytest.mark.parametrize("refill,K,B", [(0, 1, 1), (75, 1, 1), (90, 3, 1), (90, 4, 2)])
def test_trace_fork_is_result_preserving(gpu, scene_small, refill, K, B):
    """trace_fork = 1 (kernels_wavefront.hip launch_wavefront: the bounce-0 shadow walk and finish on a side stream
    beside the bounce-1 closest-hit walk) gives the serial launch order's bits: one-ray-per-lane and lane-refill
    kernels, frames in flight on several streams (each with its own side stream) and batched draws, moving camera."""
    gl = gpu
    W, H = 96, 64
    outs = []
    for fork in (0, 1):
        r = _renderer(scene_small, W, H, mode="fast", run_taa=False, run_output=False, frames_in_flight=K,
                      trace_batch=B)
        r.pass_path_tracing.set_uniform_int("trace_refill", refill)
        r.pass_path_tracing.set_uniform_int("trace_fork", fork)
        got = []
        for f in range(K + 3):
            r.camera.orbit(1.0, 0.0)
            r.frame()
            if f % 2:
                got.append({k: gl.readback(r.planes()[k]) for k in ("color", "emission", "albedo")})
        outs.append(got)
        r.close()
    for a, b in zip(*outs):
        for k in a:
            assert np.array_equal(a[k].view(np.uint32), b[k].view(np.uint32)), k


def test_wavefront_equals_megakernel(gpu, scene_small):
    """The staged (wavefront) path tracer and the single-kernel form give identical bits."""
    gl = gpu
    W, H = 96, 64
    outs = []
    for kern in (0, 1):
        r = _renderer(scene_small, W, H, mode="fast", run_taa=False, run_output=False)
        r.pass_path_tracing.set_uniform_int("pt_kernel", kern)
        for _ in range(2):
            r.frame()
        outs.append({k: gl.readback(r.planes()[k]) for k in ("color", "emission", "albedo")})
    for k in outs[0]:
        assert np.array_equal(outs[0][k], outs[1][k]), k


@pytest.mark.parametrize("W,H,stride,cap", [(96, 64, 3, 0), (100, 70, 4, 0), (96, 64, 3, 16)])
def test_tile_subsets_compose_to_full_frame(gpu, scene_small, W, H, stride, cap):
    """tile_stride / tile_offset: each subset writes exactly its 16x16 tiles (others keep their contents) and
    the subsets of one frame together give the full-frame bits (ragged edge tiles included). The primaries of a subset
    are rasterised by tile-binned leaves like a whole band's (the bins cover every tile, the subset's tiles run);
    cap = 16: a leaf-pair list too small for the frame, so every subset overflows, walks its pixels and must clear
    the tile counts of the whole band (not only its own tiles) for the next subset's binning."""
    gl = gpu
    a = _renderer(scene_small, W, H, mode="fast", run_taa=False, run_output=False)
    a.frame()
    want = {k: gl.readback(a.planes()[k]) for k in ("color", "emission", "albedo")}
    b = _renderer(scene_small, W, H, mode="fast", run_taa=False, run_output=False)
    pt = b.pass_path_tracing
    pt.set_uniform_int("raster_pair_cap", cap)
    pt.set_uniform_int("tile_stride", stride)
    pt.set_uniform_int("tile_offset", 0)
    b.frame()
    ntx = (W + 15) // 16
    ty, tx = np.meshgrid(np.arange(H) // 16, np.arange(W) // 16, indexing="ij")
    owner = (ty * ntx + tx) % stride
    got = gl.readback(b.planes()["color"])
    assert np.array_equal(got[owner == 0], want["color"][owner == 0])
    assert not got[owner != 0].any()                     # zero-initialised planes, untouched
    b.camera.frameCounter -= 1                           # the same frame again, the other subsets
    for off in range(1, stride):
        pt.set_uniform_int("tile_offset", off)
        b._path_trace()
    b.camera.frameCounter += 1
    for k, v in want.items():
        assert np.array_equal(gl.readback(b.planes()[k]), v), k
    pt.set_uniform_int("tile_offset", stride)
    with pytest.raises(Exception):
        b._path_trace()
    a.close()
    b.close()


def test_merged_environment_equals_two_fetches(gpu, scene_small):
    """hdr_merge (default 1): the NEE's radiance and pdf at one direction (path_tracing.frag:813-832) fetched from one
    merged texture (hdrMap's .xyz beside hdrCache's .z) give the bits of the two separate fetches; a new environment
    upload rebuilds the merged copy."""
    gl = gpu
    W, H = 64, 48
    outs = []
    for merge in (0, 1):
        r = _renderer(scene_small, W, H, mode="fast", run_taa=False, run_output=False)
        r.pass_path_tracing.set_uniform_int("hdr_merge", merge)
        r.frame()
        first = gl.readback(r.planes()["color"])
        gl.upload_rgb32f(r.hdrMap, scene_small.hdr[::-1].copy())  # a different environment: the merged copy follows
        r.frame()
        outs.append((first, gl.readback(r.planes()["color"])))
        r.close()
    assert np.array_equal(outs[0][0], outs[1][0]) and np.array_equal(outs[0][1], outs[1][1])
    assert not np.array_equal(outs[1][0], outs[1][1])


def test_merged_environment_rebuilds_with_frames_in_flight(gpu, scene_small):
    """The merged environment rebuilt twice (a new upload, then the first environment again) with four frames in flight
    on four streams: a rebuild writes a retired buffer once its readers' events have completed, or a new one, and the
    draws wait for the merge on their own streams (no device-wide wait); every frame equals the two-fetch path's."""
    import torch

    gl = gpu
    W, H = 64, 48
    envs = (scene_small.hdr, scene_small.hdr[::-1].copy())
    outs = []
    for merge in (0, 1):
        r = _renderer(scene_small, W, H, mode="fast", run_taa=False, run_output=False, frames_in_flight=4)
        r.pass_path_tracing.set_uniform_int("hdr_merge", merge)  # (every frame slot's pass)
        got = []
        for env in (1, 0, 1):
            for _ in range(5):
                r.frame()
            got.append(gl.readback(r.planes()["color"]))
            torch.cuda.synchronize()  # (GL orders an upload after the draws; here the host does)
            gl.upload_rgb32f(r.hdrMap, envs[env])
        r.close()
        outs.append(got)
    for a, b in zip(*outs):
        assert np.array_equal(a, b)
    assert not np.array_equal(outs[1][0], outs[1][1])


def test_fast_driver_equals_reference_driver(gpu, scene_small):
    """Pointer-swapped fast driver == main.cpp call sequence with copies, bit for bit."""
    gl = gpu
    W = H = 64
    a = _renderer(scene_small, W, H, mode="reference", run_taa=True, run_output=True)
    b = _renderer(scene_small, W, H, mode="fast", run_taa=True, run_output=True)
    for f in range(3):
        if f == 2:
            a.camera.orbit(1.0, 0.0)
            b.camera.orbit(1.0, 0.0)
        a.frame()
        b.frame()
        pa, pb = _readback(gl, a), _readback(gl, b)
        for key in ("color", "reproj_illum", "variance", "atrous", "modulate", "final", "output"):
            assert np.array_equal(pa[key], pb[key]), (f, key)


def test_debug_views_feed_the_output_pass(gpu, scene_small):
    """main.cpp:558-586: each debug view routes its plane through the output tonemap; switching views restarts
    the frame counter and toggles accumulation (gui_config.h:37-45), in both drivers identically."""
    gl = gpu
    W, H = 48, 40
    a = _renderer(scene_small, W, H, mode="reference", run_taa=True, run_output=True)
    b = _renderer(scene_small, W, H, mode="fast", run_taa=True, run_output=True)
    src = {"path_tracing_pic_1spp": "color", "svgf_reprojected_pic": "reproj_illum", "svgf_variance_pic": "variance",
           "svgf_atrous_pic": "atrous", "svgf_modulate_pic": "modulate", "taa_pic": "final", "final_pic": "final",
           "accumulate_color": "color"}
    for view, key in src.items():
        for r in (a, b):
            r.camera.frameCounter = 7
            r.set_view(view)
            assert r.camera.frameCounter == 0 and r.cfg.accumulate_color == (view == "accumulate_color")
            r.frame()
        pa, pb = _readback(gl, a), _readback(gl, b)
        want = O.output(pa[key])
        _cmp(f"{view}/output", pa["output"], want, tol=1e-6)
        assert np.array_equal(pa["output"].view(np.uint32), pb["output"].view(np.uint32)), view
    a.close()
    b.close()


@pytest.mark.parametrize("K", [1, 2])
def test_accumulate_fast_equals_reference(gpu, scene_small, K):
    """Accumulate mode (path_tracing.frag:1116-1119, lastFrame = last frame's colour): the fast driver's slot
    alternation (and, with frames in flight, front ends chained on the previous colour) gives the reference
    driver's bits, through static frames (running mean) and a camera move (frameCounter reset, camera.h:71)."""
    from ptsvgf.camera import parameter_config

    gl = gpu
    cfg = parameter_config()
    cfg.accumulate_color = True
    W, H = 64, 48
    a = _renderer(scene_small, W, H, config=cfg, mode="reference", run_taa=True, run_output=True)
    b = _renderer(scene_small, W, H, config=cfg, mode="fast", run_taa=True, run_output=True, frames_in_flight=K)
    for f in range(5):
        for r in (a, b):
            if f == 3:
                r.camera.orbit(1.0, 0.0)
            r.frame()
        pa, pb = _readback(gl, a), _readback(gl, b)
        for key in ("color", "modulate", "final", "output"):
            assert np.array_equal(pa[key].view(np.uint32), pb[key].view(np.uint32)), (f, key)
    a.close()
    b.close()


@pytest.mark.parametrize("K,lag,B", [(2, 0, 1), (3, 0, 1), (3, 1, 1), (4, 3, 1), (4, 0, 2), (4, 3, 4), (8, 0, 8)])
def test_frames_in_flight_equal_serial(gpu, scene_small, K, lag, B):
    """K frames in flight (front ends on K streams, SVGF chain on a back-end stream; with back_lag the back end
    issued `lag` frames behind the front end; with trace_batch B the path tracers of B frames drawn as one batch
    whose traversal launches trace all their rays) give the serial fast driver's bits: per frame (read back after
    each frame: a partial batch is drawn) and after K+3 frames issued without any host wait (moving camera, so
    every frame's inputs differ)."""
    gl = gpu
    W, H = 96, 64
    kw = dict(mode="fast", run_taa=True, run_output=True)
    a = _renderer(scene_small, W, H, **kw)
    b = _renderer(scene_small, W, H, frames_in_flight=K, back_lag=lag, trace_batch=B, **kw)
    keys = ("normal_depth", "color", "albedo", "reproj_illum", "variance", "atrous", "modulate", "final", "output")
    for f in range(K + 2):
        for r in (a, b):
            if f >= 2:
                r.camera.orbit(1.0, 0.0)
            r.frame()
        pa, pb = _readback(gl, a), _readback(gl, b)
        for key in keys:
            assert np.array_equal(pa[key].view(np.uint32), pb[key].view(np.uint32)), (f, key)
    for f in range(K + 3):  # no readback in between: the streams overlap frames
        for r in (a, b):
            r.camera.orbit(1.0, 0.0)
            r.frame()
    pa, pb = _readback(gl, a), _readback(gl, b)
    for key in keys:
        assert np.array_equal(pa[key].view(np.uint32), pb[key].view(np.uint32)), ("overlapped", key)
    a.close()
    b.close()


def test_host_pace_equals_serial(gpu, scene_small):
    """host_pace (the host waits for frame f - K's SVGF before issuing frame f) changes only when the host issues:
    the frames are the serial driver's bits, moving camera, no readback in between."""
    gl = gpu
    W, H = 96, 64
    kw = dict(mode="fast", run_taa=False, run_output=False)
    a = _renderer(scene_small, W, H, **kw)
    b = _renderer(scene_small, W, H, frames_in_flight=3, host_pace=True, **kw)
    for _ in range(8):
        for r in (a, b):
            r.camera.orbit(1.0, 0.0)
            r.frame()
    pa, pb = _readback(gl, a), _readback(gl, b)
    for key in ("color", "modulate", "atrous"):
        assert np.array_equal(pa[key].view(np.uint32), pb[key].view(np.uint32)), key
    a.close()
    b.close()


def test_fast_atrous_within_tolerance(gpu, scene_small):
    """Production a-trous (hardware exp2/log2) vs the exact oracle on real frame data."""
    gl = gpu
    W = H = 96
    r = _renderer(scene_small, W, H, mode="reference", atrous_exact=False, run_taa=False, run_output=False)
    ref = O.OracleFrameLoop(scene_small, W, H)
    for f in range(2):
        r.frame()
        want = ref.frame()
    got = _readback(gl, r)
    for key in ("atrous", "modulate"):
        _cmp(key, got[key], want[key], rel=True)


@pytest.mark.parametrize("mode", ["reference", "fast"])
def test_taa_and_output_match_oracle(gpu, scene_small, mode):
    """taa.frag + output_pass.frag under an orbiting camera: the TAA history (last_taa_color)
    goes through save_frame_data in the reference driver and a ping-pong pair in the fast driver."""
    gl = gpu
    W, H = 80, 64
    r = _renderer(scene_small, W, H, mode=mode, atrous_exact=True, run_taa=True, run_output=True)
    ref = O.OracleFrameLoop(scene_small, W, H, run_taa=True, run_output=True)
    for f in range(4):
        if f >= 2:
            r.camera.orbit(1.5, -0.5)
            ref.camera.orbit(1.5, -0.5)
        r.frame()
        want = ref.frame()
        got = _readback(gl, r)
        for key in ("modulate", "final", "output"):
            _cmp(f"{mode}/f{f}/{key}", got[key], want[key], rel=True)


def test_full_size_4k_properties(gpu, scene_bench):
    """At the bench size (3840x2160, the bench scene) the oracle is too slow, so size-independent properties:
    the wavefront path tracer (compacted ray lists at their largest, cost-ordered tiles, shadow trees) gives
    the megakernel's bits, and 4 frames in flight give the serial driver's bits after a moving-camera run."""
    gl = gpu
    W, H = 3840, 2160
    keys = ("color", "emission", "albedo")
    outs = []
    for kern in (0, 1):
        r = _renderer(scene_bench, W, H, mode="fast", aspect_corrected=True, run_taa=False, run_output=False)
        r.pass_path_tracing.set_uniform_int("pt_kernel", kern)
        r.frame()
        outs.append({k: gl.readback(r.planes()[k]) for k in keys})
        r.close()
    for k in keys:
        assert np.array_equal(outs[0][k].view(np.uint32), outs[1][k].view(np.uint32)), k
    del outs
    planes = []
    for K in (1, 4):
        r = _renderer(scene_bench, W, H, mode="fast", aspect_corrected=True, run_taa=False, run_output=False,
                      frames_in_flight=K)
        for _ in range(6):
            r.camera.orbit(1.0, 0.0)
            r.frame()
        planes.append({k: gl.readback(r.planes()[k]) for k in ("color", "atrous", "modulate")})
        r.close()
    for k in planes[0]:
        assert np.array_equal(planes[0][k].view(np.uint32), planes[1][k].view(np.uint32)), k


@pytest.mark.parametrize("mode,K", [("reference", 1), ("fast", 1), ("fast", 3)])
def test_accumulate_matches_oracle(gpu, scene_small, mode, K):
    """Accumulate mode against the oracle (path_tracing.frag:1116-1119: color = mix(lastFrame, color,
    1/(frameCounter+1)), lastFrame = last_acc_color refreshed by save_frame_data, main.cpp:546-553): a running mean
    over static frames, then a camera move (frameCounter reset to 0, camera.h:71, so the mean restarts), then more
    static frames. The accumulated colour is bit-exact; the SVGF chain that consumes it within the tolerance."""
    from ptsvgf.camera import parameter_config

    gl = gpu
    cfg = parameter_config()
    cfg.accumulate_color = True
    W, H = 64, 48
    r = _renderer(scene_small, W, H, config=cfg, mode=mode, atrous_exact=True, run_taa=False, run_output=False,
                  frames_in_flight=K)
    ref = O.OracleFrameLoop(scene_small, W, H, cfg, run_taa=False)
    for f in range(6):
        if f == 3:
            r.camera.orbit(1.0, 0.5)
            ref.camera.orbit(1.0, 0.5)
        r.frame()
        want = ref.frame()
        got = _readback(gl, r)
        if f == 2:
            acc2 = want["color"]
        ex = _cmp(f"{mode}/K{K}/f{f}/color", got["color"], want["color"])
        assert ex == 1.0, f"accumulated colour is not bit-exact ({ex})"
        for key in ("reproj_illum", "variance", "atrous", "modulate"):
            _cmp(f"{mode}/K{K}/f{f}/{key}", got[key], want[key], rel=True)
    # the mean really accumulates: frame 2's accumulated colour is not frame 2's own 1-spp colour
    single = O.OracleFrameLoop(scene_small, W, H, run_taa=False)
    for _ in range(3):
        one = single.frame()
    assert not np.array_equal(one["color"], acc2)
    r.close()


@pytest.mark.parametrize("scene_name", ["scene_small", "scene_cornell", "scene_nan"])
def test_lane_refill_is_result_preserving(gpu, scene_name, request):
    """trace_refill=100 / 75 (list-driven traversal waves hand the next list items to their idle lanes, for all of
    each list / its first 75 %) gives the
    one-ray-per-thread kernels' bits and traces the same rays. Visit counts may differ by a few: a lane holding a
    postponed leaf keeps descending while other lanes of its wave still look for one (while-while), and the wave
    a ray shares differs between the two forms; the verdicts and hits do not depend on it."""
    gl = gpu
    scene = request.getfixturevalue(scene_name)
    W, H = 96, 64
    outs, stats = [], []
    for refill in (100, 75, 0):
        r = _renderer(scene, W, H, mode="fast", run_taa=False, run_output=False)
        r.pass_path_tracing.set_uniform_int("trace_refill", refill)
        r.pass_path_tracing.set_uniform_int("wide_bvh", 0)  # visit counts compare on one tree shape
        r.frame()
        stats.append(r.trace_stats())
        outs.append({k: gl.readback(r.planes()[k]) for k in ("color", "emission", "albedo")})
        r.close()
    for o, st in zip(outs[:2], stats[:2]):
        for k in o:
            assert np.array_equal(o[k].view(np.uint32), outs[2][k].view(np.uint32)), k
        # the shadow split (wf_shadow_stats) counts verdicts: the same in every form
        for k in ("primary_rays", "bounce_rays", "shadow_rays", "shadow_point_rays", "shadow_occluded"):
            assert st[k] == stats[2][k], (k, stats)
        assert st["shadow_occluded"] <= st["shadow_rays"] and st["shadow_point_rays"] <= st["shadow_rays"], st
        for k in ("shadow_visits", "bounce_visits"):
            assert abs(st[k] - stats[2][k]) <= 0.01 * stats[2][k], (k, stats)


@pytest.mark.parametrize("scene_name", ["scene_small", "scene_cornell", "scene_nan"])
def test_wide_tree_is_result_preserving(gpu, scene_name, request):
    """The 4-wide form of the any-hit tree (pack_wide; wide_bvh = 1, the default) gives the binary walks' bits: lane
    refill with 4 frames in flight, a moving camera, a tiny LDS stack budget is not needed here (overflows and exact
    ties go to the cooperative walk, which the deep-tree tests exercise). Fewer node visits than the binary tree."""
    gl = gpu
    scene = request.getfixturevalue(scene_name)
    W, H = 96, 64
    outs, stats = [], []
    for wide in (1, 0):
        r = _renderer(scene, W, H, mode="fast", run_taa=False, run_output=False, frames_in_flight=4)
        r.pass_path_tracing.set_uniform_int("wide_bvh", wide)
        frames = []
        for f in range(5):
            if f == 3:
                r.camera.orbit(2.0, 1.0)
            r.frame()
            frames.append({k: gl.readback(r.planes()[k]) for k in ("color", "emission", "albedo", "modulate")})
        stats.append(r.trace_stats())
        outs.append(frames)
        r.close()
    for fw, fb in zip(*outs):
        for k in fw:
            assert np.array_equal(fw[k].view(np.uint32), fb[k].view(np.uint32)), k
    for k in ("primary_rays", "bounce_rays", "shadow_rays", "shadow_point_rays", "shadow_occluded"):
        assert stats[0][k] == stats[1][k], (k, stats)
    print("visits wide / binary:", {k: (stats[0][k], stats[1][k]) for k in ("bounce_visits", "shadow_visits")})


def test_far_eye_walks_reference_tree(gpu, scene_small):
    """the fine leaf boxes (capi.hip refine_leaves) are padded for ray origins within kFineEyeReach = 64 x
    the scene's largest vertex coordinate. An eye beyond that (here 200 units from a unit-sized scene) makes pt_params
    walk the reference tree: the default settings then give exactly the bits of the reference-tree walk
    (closest_tree = 0, shadow_tree = 0), for a camera both inside and far outside the reach."""
    gl = gpu
    W, H = 96, 64
    for r_dis in (2.0, 200.0):
        outs = []
        for ref_tree in (0, 1):
            r = _renderer(scene_small, W, H, mode="fast", run_taa=False, run_output=False)
            r.camera.r_dis = np.float32(r_dis)
            r.camera.dirty = True
            if ref_tree:
                r.pass_path_tracing.set_uniform_int("closest_tree", 0)
                r.pass_path_tracing.set_uniform_int("shadow_tree", 0)
            for _ in range(2):
                r.frame()
            outs.append({k: gl.readback(r.planes()[k]) for k in ("color", "emission", "albedo")})
            r.close()
        for k in outs[0]:
            assert np.array_equal(outs[0][k].view(np.uint32), outs[1][k].view(np.uint32)), (r_dis, k)


@pytest.mark.parametrize("W,H,moves", [(96, 64, [(2.0, 0.5), (-3.0, 1.0), (4.0, -2.0)]), (200, 120, [(1.0, 0.0)] * 3)])
def test_reproject_block_fetch_equals_per_tap(gpu, scene_small, W, H, moves):
    """The reprojection's 3x3 block fetch (reproj_block = 1, the default: the four history taps' texels loaded once per
    plane) against lin() per tap (reproj_block = 0): the same texels with the same weights, so the same bits, through
    camera moves (non-zero motion, disocclusions, the 3x3 fallback) and the frame edges."""
    gl = gpu
    out = []
    for block in (0, 1):
        r = _renderer(scene_small, W, H, mode="fast", run_taa=False, run_output=False)
        for p in r.reproject:
            p.set_uniform_int("reproj_block", block)
        planes = []
        for mv in [None] + moves:
            if mv:
                r.camera.orbit(*mv)
            r.frame()
            pl = r.planes()
            planes.append({k: gl.readback(pl[k]) for k in ("reproj_illum", "reproj_moments", "modulate")})
        r.close()
        out.append(planes)
    for f, (a, b) in enumerate(zip(*out)):
        for k in a:
            assert np.array_equal(a[k].view(np.uint32), b[k].view(np.uint32)), (f, k)


def test_renderer_streams_distinct_and_recycled(gpu, scene_small):
    """Frames in flight run on the renderer's own queues: distinct within a renderer (torch's stream pool hands its 32
    streams out round-robin, so plain torch.cuda.Stream() would alias after 32), given back on close and reused by
    the next renderer (renderer.acquire_stream)."""
    r = _renderer(scene_small, 32, 24, frames_in_flight=4)
    mine = [s.cuda_stream for s in r._streams] + [r._back.cuda_stream]
    assert len(set(mine)) == len(mine)
    r.frame()
    r.flush()
    r.close()
    r2 = _renderer(scene_small, 32, 24, frames_in_flight=4)
    again = [s.cuda_stream for s in r2._streams] + [r2._back.cuda_stream]
    assert set(again) == set(mine)
    r2.frame()
    r2.flush()
    r2.close()


@pytest.mark.parametrize("K", [1, 3])
def test_fused_modulate_equals_modulate_pass(gpu, scene_small, K):
    """The last a-trous iteration with the modulate fused into its epilogue (Renderer(fuse_modulate=True), the
    default) against the separate modulate pass: every plane identical, bit for bit, over frames with motion."""
    from ptsvgf.camera import parameter_config

    W, H = 96, 64
    out = {}
    for fuse in (False, True):
        r = _renderer(scene_small, W, H, config=parameter_config(), mode="fast", run_taa=True, run_output=True,
                      frames_in_flight=K, fuse_modulate=fuse)
        frames = []
        for i in range(4):
            r.camera.orbit(2.0, 0.5)
            r.frame()
            r.flush()
            frames.append(_readback(gpu, r))
        r.close()
        out[fuse] = frames
    for a, b in zip(out[False], out[True]):
        assert a.keys() == b.keys()
        for k in a:
            assert np.array_equal(a[k].view(np.uint32), b[k].view(np.uint32)), k


def test_cu_masked_stream_same_bits(gpu, scene_small):
    """pt_stream_create_cu_masked: frames drawn on a stream kept off 32 CUs (and the trace_fork side stream, which
    inherits the mask) give the default stream's bits; pt_stream_destroy releases it."""
    import ctypes as C

    import torch

    from ptsvgf._lib import check, pt
    from ptsvgf.renderer import masked_stream, reserved_cus

    gl = gpu
    W, H = 64, 48
    n = C.c_int()
    check(pt().pt_device_cus(C.byref(n)))
    assert n.value >= 64
    excl = reserved_cus(n.value, 32)
    assert len(excl) == 32 and len({i // (n.value // 8) for i in excl}) == 8
    outs = []
    for masked in (False, True):
        st, h = masked_stream(excl) if masked else (torch.cuda.current_stream(), None)
        with torch.cuda.stream(st):
            r = _renderer(scene_small, W, H, mode="fast", run_taa=False, run_output=False)
            r.pass_path_tracing.set_uniform_int("trace_fork", 1)
            for f in range(3):
                if f == 2:
                    r.camera.orbit(1.0, 0.0)
                r.frame()
            outs.append({k: gl.readback(r.planes()[k]) for k in ("color", "atrous", "modulate")})
            r.close()
        torch.cuda.synchronize()
        if h is not None:
            check(pt().pt_stream_destroy(h))
    for k in outs[0]:
        assert np.array_equal(outs[0][k], outs[1][k]), k


def test_priority_stream_same_bits(gpu, scene_small):
    """pt_stream_create_priority: frames drawn on a low-priority stream (and its trace_fork side stream, which takes
    the draw stream's priority) give the default stream's bits; out-of-range priorities clamp."""
    import ctypes as C

    import torch

    from ptsvgf._lib import check, pt
    from ptsvgf.renderer import priority_stream

    gl = gpu
    lo, hi = C.c_int(), C.c_int()
    check(pt().pt_stream_priority_range(C.byref(lo), C.byref(hi)))
    assert hi.value <= 0 <= lo.value
    W, H = 64, 48
    outs = []
    for prio in (None, lo.value + 5):  # clamped to the least priority
        st, h = priority_stream(prio) if prio is not None else (torch.cuda.current_stream(), None)
        with torch.cuda.stream(st):
            r = _renderer(scene_small, W, H, mode="fast", run_taa=False, run_output=False)
            r.pass_path_tracing.set_uniform_int("trace_fork", 1)
            for f in range(3):
                if f == 2:
                    r.camera.orbit(1.0, 0.0)
                r.frame()
            outs.append({k: gl.readback(r.planes()[k]) for k in ("color", "atrous", "modulate")})
            r.close()
        torch.cuda.synchronize()
        if h is not None:
            check(pt().pt_stream_destroy(h))
    for k in outs[0]:
        assert np.array_equal(outs[0][k], outs[1][k]), k


@pytest.mark.parametrize("scene_name", ["scene_small", "scene_cornell"])
def test_strided_launch_grids_are_result_preserving(gpu, scene_name, request):
    """The refill traversal launches with a grid far below their waves (uniform refill_grid = 3 blocks: every wave
    walks many static chunks in turn, WaveQueue::grab) and the list-driven shade / finish with 8 blocks striding over
    256-item chunks (uniform list_grid) give the default grids' bits, through a camera move and frames in flight."""
    gl = gpu
    scene = request.getfixturevalue(scene_name)
    W, H = 96, 64
    outs = []
    for grid in (0, 3):
        r = _renderer(scene, W, H, mode="fast", run_taa=False, run_output=False, frames_in_flight=2)
        r.pass_path_tracing.set_uniform_int("refill_grid", grid)
        r.pass_path_tracing.set_uniform_int("list_grid", 8 if grid else 0)
        frames = []
        for f in range(4):
            if f == 2:
                r.camera.orbit(2.0, 1.0)
            r.frame()
            frames.append({k: gl.readback(r.planes()[k]) for k in ("color", "emission", "albedo", "modulate")})
        outs.append(frames)
        r.close()
    for a, b in zip(*outs):
        for k in a:
            assert np.array_equal(a[k].view(np.uint32), b[k].view(np.uint32)), k
