"""A/B timing of the a-trous variants on real 4K frame data, default and surface-dominated views.

For each view: render 3 frames, then time every variant x step as 20 back-to-back launches between two HIP
events on the library stream (no per-launch sync), interleaved over ROUNDS rounds; report the median per-launch
time and the algorithmic (52 B/px) fraction of 8 TB/s. The variants' outputs are compared bit for bit.
usage: python tools/bench_atrous.py [variant ...]   (variants: 0 tile, 1 generic, 2 step; default 0 2)
A variant may carry extra int uniforms: 0:atrous_tile_flags=0"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "path-tracing-svgf_amd"))
sys.path.insert(0, REPO)
import numpy as np
import torch

from bench import VIEWS
from ptsvgf import gl
from ptsvgf._lib import check, pt
from ptsvgf.camera import parameter_config
from ptsvgf.gl import GL_TEXTURE_2D, RenderPass
from ptsvgf.renderer import Renderer, _prog
from ptsvgf.scene import build_scene

W, H = int(os.environ.get("W", 3840)), int(os.environ.get("H", 2160))
VARIANTS = sys.argv[1:] or ["0", "2"]


def select(ap, spec):
    """Set atrous_variant and the spec's extra uniforms (reset to 0 first so variants do not leak into each other)."""
    v, *kv = spec.split(":")
    for name in ("atrous_tile_flags",):
        ap.set_uniform_int(name, {"atrous_tile_flags": 1}.get(name, 0))
    ap.set_uniform_int("atrous_variant", int(v))
    for item in kv:
        name, val = item.split("=")
        ap.set_uniform_int(name, int(val))
torch.cuda.set_device(0)
gl.init(0)
check(pt().pt_set_stream(torch.cuda.current_stream().cuda_stream))
scene = build_scene("table_clock_plant")
for view in ("default", "surface"):
    r = Renderer(scene, W, H, parameter_config(), mode="fast", aspect_corrected=True, run_taa=False, run_output=False)
    if VIEWS[view]:
        for k, v in VIEWS[view].items():
            setattr(r.camera, k, np.array(v, np.float32) if isinstance(v, tuple) else np.float32(v))
        r.camera.dirty = True
    for _ in range(3):
        r.frame()
    torch.cuda.synchronize()
    pl = r.planes()
    out = gl.getTextureRGB32F(W, H)
    ap = RenderPass(_prog("svgf_Atrous.frag"), W, H)
    ap.colorAttachments.append(out)
    ap.bindData(False)
    ap.set_uniform_float("gPhiColor", 4.0)
    ap.set_uniform_float("gPhiNormal", 128.0)
    ap.set_texture_uniform(GL_TEXTURE_2D, pl["normal_depth"], "gNormalAndLinearZ")
    ap.set_texture_uniform(GL_TEXTURE_2D, pl["fwidth"], "gNormalDepthFwidth")
    ap.set_texture_uniform(GL_TEXTURE_2D, pl["variance"], "gIllumination")
    surf = float(np.mean(gl.readback(pl["normal_depth"])[..., 3] != 1.0))
    res = {}
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for rnd in range(int(os.environ.get("ROUNDS", 5))):
        for v in VARIANTS:
            select(ap, v)
            for step in (1, 2, 4, 8, 16):
                ap.set_uniform_int("gStepSize", step)
                ap.draw()
                e0.record()
                for _ in range(20):
                    ap.draw()
                e1.record()
                e1.synchronize()
                res.setdefault((v, step), []).append(e0.elapsed_time(e1) / 20)
    for (v, step), ts in sorted(res.items()):
        med = float(np.median(ts))
        print(json.dumps(dict(view=view, surface=round(surf, 3), variant=v, step=step, us=round(med * 1e3, 1),
                              frac=round(52 * W * H / (med * 1e-3) / 8e12, 3))), flush=True)
    for v in VARIANTS:
        print(json.dumps(dict(view=view, variant=v, mean_us=round(float(np.mean(
            [np.median(res[(v, s)]) for s in (1, 2, 4, 8, 16)])) * 1e3, 1))), flush=True)
    outs = {}
    for v in VARIANTS:
        for step in (1, 2, 4, 8, 16):
            select(ap, v)
            ap.set_uniform_int("gStepSize", step)
            ap.draw()
            outs[(v, step)] = gl.readback(out)
    for v in VARIANTS[1:]:
        same = all(np.array_equal(outs[(v, s)].view(np.uint32), outs[(VARIANTS[0], s)].view(np.uint32))
                   for s in (1, 2, 4, 8, 16))
        print(f"{view}: variant {v} bit-identical to variant {VARIANTS[0]}: {same}", flush=True)
    ap.destroy()
    gl.destroy_texture(out)
    r.close()
gl.shutdown()
