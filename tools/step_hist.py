"""Per-pixel traversal steps of one 4K frame (investigation build: PTSVGF_LIB_DIR=.../lib_exp/stepmax, compiled
with -DPT_STEP_MAX so the row-cost probe records each pixel's largest node+triangle visit count over all its
rays). Prints percentiles and the worst pixels. usage: python tools/step_hist.py"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "path-tracing-svgf_amd"))
import numpy as np
import torch

from ptsvgf import gl
from ptsvgf.camera import parameter_config
from ptsvgf.renderer import Renderer
from ptsvgf.scene import build_scene

W, H = 3840, 2160
torch.cuda.set_device(0)
gl.init(0)
r = Renderer(build_scene("table_clock_plant"), W, H, parameter_config(), mode="fast", aspect_corrected=True,
             run_taa=False, run_output=False)
r.frame()
c = torch.zeros(W * H, dtype=torch.int32, device="cuda")
r.pass_path_tracing.set_row_cost(c.data_ptr())
r.frame()
torch.cuda.synchronize()
s = c.cpu().numpy().reshape(H, W)
print("percentiles 50/90/99/99.9/99.99/max:", [int(np.percentile(s, q)) for q in (50, 90, 99, 99.9, 99.99)],
      int(s.max()))
idx = np.argsort(s.ravel())[::-1][:12]
for i in idx:
    print("pixel", (i % W, i // W), "steps", int(s.ravel()[i]))
# per 64-px wave (8x8 tiles as wf_primary) max vs mean
t = s.reshape(H // 8, 8, W // 8, 8).max(axis=(1, 3))
print("8x8 tile max percentiles 50/99/max:", [int(np.percentile(t, q)) for q in (50, 99)], int(t.max()))
rows = s.max(axis=1)
print("row max by 270-row band:", [int(rows[i:i + 270].max()) for i in range(0, H, 270)])
np.save(os.path.join(REPO, "gpurun_out", "steps.npy"), np.minimum(s, 65535).astype(np.uint16))
gl.shutdown()
