"""Kernel-level cost of a tile-subset path tracer (the tile shard's per-rank draw): FRAMES draws of the subset
k * STRIDE + OFFSET of the 4K bench frame, one at a time (K = 1), wall-clock per draw; run it under
rocprofv3 --kernel-trace --stats to see which launches the subset pays for whole-frame sizes.
usage: STRIDE=8 OFFSET=0 FRAMES=20 python tools/pt_subset_prof.py [W] [H]"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "path-tracing-svgf_amd"))
import torch

from ptsvgf import gl
from ptsvgf.camera import parameter_config
from ptsvgf.renderer import Renderer
from ptsvgf.scene import build_scene

W = int(sys.argv[1]) if len(sys.argv) > 1 else 3840
H = int(sys.argv[2]) if len(sys.argv) > 2 else 2160
STRIDE = int(os.environ.get("STRIDE", "8"))
OFFSET = int(os.environ.get("OFFSET", "0"))
FRAMES = int(os.environ.get("FRAMES", "20"))

torch.cuda.set_device(0)
gl.init(0)
from ptsvgf._lib import check, pt  # noqa: E402

check(pt().pt_set_stream(torch.cuda.current_stream().cuda_stream))
r = Renderer(build_scene("table_clock_plant"), W, H, parameter_config(), mode="fast", aspect_corrected=True,
             run_taa=False, run_output=False)
for stride, off in ((STRIDE, OFFSET),):
    r.pass_path_tracing.set_uniform_int("tile_stride", stride)
    r.pass_path_tracing.set_uniform_int("tile_offset", off)
    for uv in filter(None, os.environ.get("PT_UNIFORMS", "").split(",")):
        k, v = uv.split("=")
        r.pass_path_tracing.set_uniform_int(k, int(v))
    for _ in range(3):
        r._path_trace()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(FRAMES):
        r._path_trace()
        r.camera.frameCounter += 1
    torch.cuda.synchronize()
    print(f"stride {stride} offset {off}: {(time.perf_counter() - t0) * 1e3 / FRAMES:.3f} ms per draw", flush=True)
r.close()
gl.shutdown()
