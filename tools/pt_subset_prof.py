"""Kernel-level cost of a tile-subset path tracer (the tile shard's per-rank draw): FRAMES draws of the subset
k * STRIDE + OFFSET of the 4K bench frame, one at a time (K = 1), wall-clock per draw; run it under
rocprofv3 --kernel-trace --stats to see which launches the subset pays for at whole-frame size. BATCH = B > 1: the
subsets of B consecutive frames drawn as one batch (pt_pass_draw_batch), as a tile-shard rank batching its frames
would; the time is reported per batch and per frame.
usage: STRIDE=8 OFFSET=0 FRAMES=20 BATCH=1 python tools/pt_subset_prof.py [W] [H]"""
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
B = int(os.environ.get("BATCH", "1"))

torch.cuda.set_device(0)
gl.init(0)
from ptsvgf._lib import check, pt  # noqa: E402

check(pt().pt_set_stream(torch.cuda.current_stream().cuda_stream))
r = Renderer(build_scene("table_clock_plant"), W, H, parameter_config(), mode="fast", aspect_corrected=True,
             run_taa=False, run_output=False, frames_in_flight=max(2, B), trace_batch=B)
r._stream_to(torch.cuda.current_stream())  # every draw on one stream: batches one after another
r.pass_path_tracing.set_uniform_int("tile_stride", STRIDE)
r.pass_path_tracing.set_uniform_int("tile_offset", OFFSET)
r.pass_path_tracing.set_uniform_int("trace_refill", 90)  # the lane-refill walks, as with frames in flight
for uv in filter(None, os.environ.get("PT_UNIFORMS", "").split(",")):
    k, v = uv.split("=")
    r.pass_path_tracing.set_uniform_int(k, int(v))


def batch():
    passes = []
    for s in range(B):
        r._use_slot(s)
        r._path_trace()  # uniforms (with trace_batch > 1 it returns before drawing)
        passes.append(r.pt_pass)
        r.camera.frameCounter += 1
    if B > 1:
        gl.draw_batch(passes)


for _ in range(3):
    batch()
torch.cuda.synchronize()
t0 = time.perf_counter()
n = max(1, FRAMES // B)
for _ in range(n):
    batch()
torch.cuda.synchronize()
ms = (time.perf_counter() - t0) * 1e3 / n
print(f"stride {STRIDE} offset {OFFSET} batch {B}: {ms:.3f} ms per draw, {ms / B:.3f} ms per frame", flush=True)
r.close()
gl.shutdown()
