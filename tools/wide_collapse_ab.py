"""One process of the 4-wide collapse A/B (capi.hip pack_wide, PTSVGF_WIDE_COLLAPSE read once per process): renders
the bench scene, prints the traversal counters of one frame (node + triangle visits per kind) and a digest of the
path tracer's planes, so two runs with PTSVGF_WIDE_COLLAPSE = 0 / 1 show the visits each tree costs and that the
bits are the same. PTSVGF_WIDE_STATS=1 also prints the tree's summed node area.
usage: PTSVGF_WIDE_COLLAPSE=1 python tools/wide_collapse_ab.py [W] [H] [view]"""
import hashlib
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "path-tracing-svgf_amd"))
import torch

from ptsvgf import gl
from ptsvgf.camera import parameter_config
from ptsvgf.renderer import Renderer
from ptsvgf.scene import build_scene


def main() -> None:
    W = int(sys.argv[1]) if len(sys.argv) > 1 else 1920
    H = int(sys.argv[2]) if len(sys.argv) > 2 else 1080
    view = sys.argv[3] if len(sys.argv) > 3 else "default"
    scene = build_scene("table_clock_plant")
    gl.init(0)
    r = Renderer(scene, W, H, parameter_config(), mode="fast", aspect_corrected=True, run_taa=False, run_output=False)
    if view == "surface":  # bench.py VIEWS["surface"]
        import numpy as np

        for k, v in dict(r_dis=0.8, upAngle=70.0, rotatAngle=180.0, move_vec=(0.4, -0.25, 0.0)).items():
            setattr(r.camera, k, np.array(v, np.float32) if isinstance(v, tuple) else np.float32(v))
        r.camera.dirty = True
    for _ in range(3):
        r.frame()
    st = r.trace_stats()
    torch.cuda.synchronize()
    h = hashlib.sha256()
    for k in ("color", "emission", "albedo"):
        h.update(gl.readback(r.planes()[k]).tobytes())
    out = {"collapse": os.environ.get("PTSVGF_WIDE_COLLAPSE", "default"),
           "treelet": os.environ.get("PTSVGF_TREELET", "default"), "view": view, "W": W, "H": H,
           "bounce_visits": st["bounce_visits"], "shadow_visits": st["shadow_visits"],
           "bounce_rays": st["bounce_rays"], "shadow_rays": st["shadow_rays"], "planes_sha256": h.hexdigest()[:16]}
    print(json.dumps(out))
    r.close()


if __name__ == "__main__":
    main()
