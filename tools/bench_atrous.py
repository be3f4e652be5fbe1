"""A/B timing of the a-trous variants on real 4K frame data (interleaved rounds, one process)."""
import os, sys, time, json
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "path-tracing-svgf_amd"))
import numpy as np
from ptsvgf import gl
from ptsvgf.gl import GL_TEXTURE_2D, RenderPass
from ptsvgf.camera import parameter_config
from ptsvgf.renderer import Renderer, _prog
from ptsvgf.scene import build_scene

W, H = int(os.environ.get("W", 3840)), int(os.environ.get("H", 2160))
gl.init(0)
scene = build_scene("table_clock_plant")
r = Renderer(scene, W, H, parameter_config(), mode="fast", aspect_corrected=True, run_taa=False, run_output=False)
for _ in range(3):
    r.frame()
gl.sync()
pl = r.planes()
out = gl.getTextureRGB32F(W, H)
ap = RenderPass(_prog("svgf_Atrous.frag"), W, H)
ap.colorAttachments.append(out)
ap.bindData(False)
ap.set_uniform_float("gPhiColor", 4.0); ap.set_uniform_float("gPhiNormal", 128.0)
ap.set_texture_uniform(GL_TEXTURE_2D, pl["normal_depth"], "gNormalAndLinearZ")
ap.set_texture_uniform(GL_TEXTURE_2D, pl["fwidth"], "gNormalDepthFwidth")
ap.set_texture_uniform(GL_TEXTURE_2D, pl["variance"], "gIllumination")
gl.set_profiling(True)
res = {}
variants = {"step": 0, "simple": 1}
for rnd in range(int(os.environ.get("ROUNDS", 5))):
    for name, v in variants.items():
        ap.set_uniform_int("atrous_variant", v)
        for step in (1, 2, 4, 8, 16):
            ap.set_uniform_int("gStepSize", step)
            ts = []
            for _ in range(10):
                ap.draw()
                ts.append(ap.last_ms())
            res.setdefault((name, step), []).extend(ts)
bytes_ = 52 * W * H
rows = []
for (name, step), ts in sorted(res.items()):
    med = float(np.median(ts))
    rows.append(dict(variant=name, step=step, median_us=round(med * 1e3, 1), min_us=round(min(ts) * 1e3, 1),
                     algo_GBs=round(bytes_ / (med * 1e-3) / 1e9, 1)))
for row in rows:
    print(json.dumps(row))
# equivalence of the two variants on this data
outs = {}
for name, v in variants.items():
    ap.set_uniform_int("atrous_variant", v); ap.set_uniform_int("gStepSize", 4); ap.draw()
    outs[name] = gl.readback(out)
d = np.abs(outs["step"] - outs["simple"]) / np.maximum(1, np.abs(outs["simple"]))
print("max rel diff step vs simple:", float(np.nanmax(d)))
gl.shutdown()
