"""Count non-finite values per pass for the a-trous variants (diagnostic)."""
import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "path-tracing-svgf_amd")); sys.path.insert(0, os.path.join(REPO, "tests"))
import numpy as np
from ptsvgf import gl
from ptsvgf.camera import parameter_config
from ptsvgf.renderer import Renderer
from ptsvgf.scene import build_scene

W, H = 64, 96
scene = build_scene("table_clock_plant", hdr_size=(256, 128), plant_leaves=40)
gl.init(0)
for name, exact, variant in (("exact", 1, 0), ("simple", 0, 1), ("step", 0, 0)):
    r = Renderer(scene, W, H, parameter_config(), mode="fast", aspect_corrected=True, run_taa=False, run_output=False,
                 atrous_exact=bool(exact))
    for p in r.atrous_to.values():
        p.set_uniform_int("atrous_variant", variant)
    for f in range(3):
        r.frame()
        pl = r.planes()
        msg = []
        for k in ("color", "albedo", "emission", "reproj_illum", "reproj_moments", "variance", "atrous", "history_illum",
                  "modulate", "normal_depth"):
            a = gl.readback(pl[k])
            n = int((~np.isfinite(a)).sum())
            if n:
                yx = np.argwhere(~np.isfinite(a).all(-1))[:3].tolist()
                msg.append(f"{k}:{n}@{yx}")
        print(name, "frame", f, " ".join(msg) or "all finite")
    if name == "step":
        a = gl.readback(pl["variance"])
        bad = np.argwhere(~np.isfinite(gl.readback(pl["atrous"])).all(-1))
        for (y, x) in bad[:3]:
            print("variance around", y, x, a[max(0, y - 2):y + 3, max(0, x - 2):x + 3].reshape(-1, 4)[:6])
gl.shutdown()
