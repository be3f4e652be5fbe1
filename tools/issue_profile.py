"""Host-side issue cost of the frame loop: cProfile over FRAMES frames issued without synchronising, so a HIP or
torch call that blocks the host (instead of queueing) shows up with its cumulative time.
usage: python tools/issue_profile.py [W] [H]   env: FIF (frames in flight, 8), FRAMES (20)"""
import cProfile
import os
import pstats
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "path-tracing-svgf_amd"))
import torch

from ptsvgf import gl
from ptsvgf.camera import parameter_config
from ptsvgf.renderer import Renderer
from ptsvgf.scene import build_scene

W = int(sys.argv[1]) if len(sys.argv) > 1 else 1920
H = int(sys.argv[2]) if len(sys.argv) > 2 else 1080
K = int(os.environ.get("FIF", "8"))
FRAMES = int(os.environ.get("FRAMES", "20"))

torch.cuda.set_device(0)
gl.init(0)
from ptsvgf._lib import check, pt  # noqa: E402

check(pt().pt_set_stream(torch.cuda.current_stream().cuda_stream))
r = Renderer(build_scene("table_clock_plant"), W, H, parameter_config(), mode="fast", aspect_corrected=True,
             run_taa=False, run_output=False, frames_in_flight=K)
for _ in range(2 * K):
    r.frame()
torch.cuda.synchronize()
prof = cProfile.Profile()
t0 = time.perf_counter()
prof.enable()
for _ in range(FRAMES):
    r.frame()
prof.disable()
issue = (time.perf_counter() - t0) / FRAMES
torch.cuda.synchronize()
wall = (time.perf_counter() - t0) / FRAMES
print(f"K={K} {W}x{H}: issue {issue * 1e3:.3f} ms/frame, wall {wall * 1e3:.3f} ms/frame")
pstats.Stats(prof).sort_stats("tottime").print_stats(12)
r.close()
gl.shutdown()
