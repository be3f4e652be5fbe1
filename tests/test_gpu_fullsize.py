"""Oracle parity at the BENCHMARKED configuration (BASELINE.json configs[1] and configs[2]).

The bench (bench.py) renders the full table+clock+plant scene (150 plant leaves,
30 633 triangles, 2048x1024 HDR) at 1920x1080 and 3840x2160, aspect-corrected,
with the fast driver (pointer-swapped history), the production LDS-tiled a-trous
(hardware exp2/log2), 4 frames in flight and every default switch of the path
tracer (primary rays bounded by the G-buffer, closest-hit rays on the SAH tree
over the reference leaves, shadow rays on the any-hit tree, cost-ordered tiles).
This test renders exactly that configuration through the C ABI and compares
every plane with the CPU oracle's frame loop (main.cpp:436-553 restated,
tests/oracle_ref.py) on the same camera path: 3 static frames (history grows,
frameCounter 0..2), then 2 orbiting frames moving both yaw and pitch (non-zero
motion, frameCounter reset, camera.h:71).

Bars (north_star: 1e-3 per-channel L-inf, fp32):
  * path-tracer outputs (color / emission / albedo): bit-exact;
  * G-buffer planes: L-inf <= 1e-5 (the ray-cast definition);
  * SVGF planes (reproject, variance, a-trous, history, modulate): L-inf <= 1e-3, relative above 1.0.
Each comparison prints max|diff| and the bit-exact share (run with -s to see them).
"""
import os
import time

import numpy as np
import pytest

import oracle_ref as O

pytestmark = pytest.mark.gpu

TOL = 1e-3
THREADS = min(16, os.cpu_count() or 1)
MOVES = [None, None, None, (1.0, 0.75), (-1.5, -1.0)]  # (yaw, pitch) degrees before the frame
PT_KEYS = ("color", "emission", "albedo")
GB_KEYS = ("world", "normal_depth", "velocity", "fwidth")
SVGF_KEYS = ("reproj_illum", "reproj_moments", "variance", "atrous", "history_illum", "modulate")


def _cmp(tag, got, want, tol, rel):
    assert got.shape == want.shape, (tag, got.shape, want.shape)
    gn, wn = np.isnan(got), np.isnan(want)
    assert np.array_equal(gn, wn), f"{tag}: NaN pattern differs ({int(gn.sum())} vs {int(wn.sum())})"
    g = np.where(gn, 0.0, got).astype(np.float64)
    w = np.where(wn, 0.0, want).astype(np.float64)
    d = np.abs(g - w)
    if rel:
        d /= np.maximum(1.0, np.abs(w))
    mx = float(d.max()) if d.size else 0.0
    exact = float(np.mean(got.view(np.uint32) == want.view(np.uint32)))
    print(f"  {tag:28s} max|diff|={mx:.3e} bit-exact={exact * 100:8.4f}%", flush=True)
    assert mx <= tol, f"{tag}: L-inf {mx} > {tol}"
    return mx, exact


@pytest.fixture(scope="module")
def scene_bench():
    from ptsvgf.scene import build_scene

    return build_scene("table_clock_plant")  # the bench scene, full size


@pytest.mark.parametrize("W,H", [(1920, 1080), (3840, 2160)])
def test_bench_configuration_matches_oracle(gpu, scene_bench, W, H):
    import torch

    from ptsvgf.camera import parameter_config
    from ptsvgf.renderer import Renderer

    gl = gpu
    cfg = parameter_config()
    # bench.py run(): the measured renderer, switch for switch
    r = Renderer(scene_bench, W, H, cfg, mode="fast", aspect_corrected=True, run_taa=False, run_output=False,
                 frames_in_flight=4)
    r.pass_path_tracing.set_uniform_int("pt_kernel", 0)
    ref = O.OracleFrameLoop(scene_bench, W, H, parameter_config(), aspect_corrected=True, threads=THREADS,
                            run_taa=False)
    worst = {}
    for f, mv in enumerate(MOVES):
        if mv:
            r.camera.orbit(*mv)
            ref.camera.orbit(*mv)
        t0 = time.perf_counter()
        r.frame()
        torch.cuda.synchronize()
        want = ref.frame()
        t1 = time.perf_counter()
        got = {k: gl.readback(v) for k, v in r.planes().items()}
        surf = float(np.mean(want["normal_depth"][..., 3] != 1.0))
        print(f"{W}x{H} frame {f} move={mv} frameCounter={ref.camera.frameCounter - 1} surface={surf * 100:.1f}% "
              f"(oracle {t1 - t0:.1f} s on {THREADS} threads)", flush=True)
        if mv:
            mo = want["velocity"][..., :2][want["normal_depth"][..., 3] != 1.0]
            print(f"  max |motion| = {np.abs(mo).max(axis=0) * (W, H)} px", flush=True)
            assert np.abs(mo).max() > 0
        for k in PT_KEYS:
            mx, ex = _cmp(f"f{f}/{k}", got[k], want[k], TOL, False)
            assert ex == 1.0, f"path-tracer plane {k} is not bit-exact at {W}x{H} frame {f} ({ex})"
            worst[k] = max(worst.get(k, 0.0), mx)
        for k in GB_KEYS:
            worst[k] = max(worst.get(k, 0.0), _cmp(f"f{f}/{k}", got[k], want[k], 1e-5, False)[0])
        for k in SVGF_KEYS:
            worst[k] = max(worst.get(k, 0.0), _cmp(f"f{f}/{k}", got[k], want[k], TOL, True)[0])
        del got, want
    print(f"{W}x{H} per-pass worst max|diff| over {len(MOVES)} frames: "
          + ", ".join(f"{k}={v:.2e}" for k, v in worst.items()), flush=True)
    r.close()
