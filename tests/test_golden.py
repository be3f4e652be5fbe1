"""Committed fixtures under tests/golden/ (generator: tools/make_golden.py).

scene_kat.json holds the reference's own host-prep known answers; oracle_frames.npz
holds oracle regression frames (parity of the GLSL passes is unpinned — see
DESIGN.md "Pinning"). The CPU test proves the oracle still reproduces the
vectors; the GPU test compares the HIP path with them directly, so the GPU box
checks against data that was produced here.
"""
import json
import os
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = os.path.join(HERE, "golden")
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "tools"))

import make_golden as G  # noqa: E402


def _frames():
    z = np.load(os.path.join(GOLDEN, "oracle_frames.npz"))
    return {k: z[k] for k in z.files}


def test_scene_kat_fixture_matches_host_prep():
    from ptsvgf.scene import SceneBuilder, material, transform
    kat = json.load(open(os.path.join(GOLDEN, "scene_kat.json")))
    models = os.path.join(os.path.dirname(HERE), "assets", "models")
    for name in ("clock", "table"):
        b = SceneBuilder()
        b.add_obj(os.path.join(models, f"{name}.obj"), material(), transform(), True, 0)
        b.build(8)
        c = b.counts()
        want = kat[name]
        assert (c["triangles"], c["nodes"], c["leaves"], c["max_depth"]) == (
            want["triangles"], want["nodes"], want["leaves"], want["depth"]), name


def test_oracle_reproduces_golden_frames():
    import oracle_ref as O
    from ptsvgf.scene import build_scene

    z = _frames()
    W, H = int(z["W"]), int(z["H"])
    scene = build_scene("table_clock_plant", **G.SCENE_ARGS)
    assert scene.counts["triangles"] == int(z["ntris"])
    loop = O.OracleFrameLoop(scene, W, H, run_taa=True, run_output=True, threads=4)
    for f in range(int(z["frames"])):
        if G.orbit(f):
            loop.camera.orbit(*G.orbit(f))
        o = loop.frame()
        for k in G.KEYS:
            np.testing.assert_array_equal(o[k], z[f"f{f}_{k}"], err_msg=f"f{f}/{k}")


@pytest.mark.gpu
def test_hip_matches_golden_frames(gpu):
    from ptsvgf.renderer import Renderer
    from ptsvgf.scene import build_scene

    gl = gpu
    z = _frames()
    W, H = int(z["W"]), int(z["H"])
    r = Renderer(build_scene("table_clock_plant", **G.SCENE_ARGS), W, H, mode="reference", atrous_exact=True,
                 run_taa=True, run_output=True)
    for f in range(int(z["frames"])):
        if G.orbit(f):
            r.camera.orbit(*G.orbit(f))
        r.frame()
        planes = r.planes()
        for k in G.KEYS:
            got, want = gl.readback(planes[k]), z[f"f{f}_{k}"]
            if k in ("color", "emission", "albedo"):
                assert np.array_equal(got, want), f"f{f}/{k}: path tracer not bit-exact"
            d = np.abs(got.astype(np.float64) - want) / np.maximum(1.0, np.abs(want))
            assert np.array_equal(np.isnan(got), np.isnan(want)), f"f{f}/{k}: NaN mismatch"
            assert np.nanmax(d) <= 1e-3, f"f{f}/{k}: {np.nanmax(d)}"
