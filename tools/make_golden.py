"""Generate tests/golden/ fixtures.

* scene_kat.json — the reference's own known answers for host scene preparation
  (counts printed by the reference's compiled host code for
  clock.obj / table.obj; transcribed, not computed here).
* oracle_frames.npz — small end-to-end frame vectors from the CPU oracle
  (G-buffer -> path tracer -> SVGF -> TAA -> output) on a fixed scene and
  camera path. These are REGRESSION vectors of the oracle (the GLSL passes are
  parity unpinned: the reference ships no GPU goldens and its GL path cannot run
  here). tests/test_golden.py checks that the oracle still reproduces them, and
  tests/test_gpu_parity.py checks the HIP path against them on the GPU box,
  where the oracle is not rebuilt.

Usage: python tools/make_golden.py
"""
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "path-tracing-svgf_amd"), os.path.join(REPO, "tests")]

GOLDEN = os.path.join(REPO, "tests", "golden")
W, H, FRAMES = 40, 32, 3
SCENE_ARGS = dict(hdr_size=(128, 64), plant_leaves=20)
KEYS = ("normal_depth", "velocity", "color", "emission", "albedo", "reproj_illum", "variance", "atrous", "modulate",
        "final", "output")


def orbit(f):
    """Camera move before frame f (frame 0 and 1 static, then orbit)."""
    return (2.0, 0.5) if f >= 2 else None


def main():
    import oracle_ref as O
    from ptsvgf.scene import build_scene

    os.makedirs(GOLDEN, exist_ok=True)
    kat = {
        "source": "SURVEY.md §8(c): reference host code output (readObj + buildBVHwithSAH, n=8)",
        "clock": {"triangles": 8265, "nodes": 3010, "leaves": 1505, "depth": 15},
        "table": {"triangles": 5184, "nodes": 2078, "leaves": 1039, "depth": 17},
        "table+clock": {"triangles": 13449, "nodes": 5098},
    }
    with open(os.path.join(GOLDEN, "scene_kat.json"), "w") as f:
        json.dump(kat, f, indent=1)

    scene = build_scene("table_clock_plant", **SCENE_ARGS)
    loop = O.OracleFrameLoop(scene, W, H, run_taa=True, run_output=True, threads=4)
    out = {"W": W, "H": H, "frames": FRAMES, "ntris": scene.counts["triangles"]}
    for fr in range(FRAMES):
        if orbit(fr):
            loop.camera.orbit(*orbit(fr))
        o = loop.frame()
        for k in KEYS:
            out[f"f{fr}_{k}"] = o[k].astype(np.float32)
    np.savez_compressed(os.path.join(GOLDEN, "oracle_frames.npz"), **out)
    print("wrote", os.path.join(GOLDEN, "oracle_frames.npz"))


if __name__ == "__main__":
    main()
