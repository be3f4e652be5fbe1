"""Is the frame loop host-bound? Per configuration: the host time to issue one frame() (no synchronisation inside
the loop; the library returns once the draws are queued, except where a frame slot's previous use must finish)
against the wall time per frame of the same loop. Issue time close to the wall time means the GPU waits on Python.
usage: python tools/host_issue.py"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["GPU_MAX_HW_QUEUES"] = os.environ.get("PTSVGF_HW_QUEUES", "16")
sys.path.insert(0, os.path.join(REPO, "path-tracing-svgf_amd"))
import torch  # noqa: E402

from ptsvgf import gl  # noqa: E402
from ptsvgf._lib import check, pt  # noqa: E402
from ptsvgf.camera import parameter_config  # noqa: E402
from ptsvgf.renderer import Renderer  # noqa: E402
from ptsvgf.scene import build_scene  # noqa: E402

torch.cuda.set_device(0)
gl.init(0)
check(pt().pt_set_stream(torch.cuda.current_stream().cuda_stream))
scene = build_scene("table_clock_plant")
for W, H, K in ((1920, 1080, 6), (1920, 1080, 1), (3840, 2160, 4)):
    check(pt().pt_set_stream(torch.cuda.current_stream().cuda_stream))
    r = Renderer(scene, W, H, parameter_config(), mode="fast", aspect_corrected=True, run_taa=False, run_output=False,
                 frames_in_flight=K)
    for _ in range(K + 5):
        r.frame()
    torch.cuda.synchronize()
    n = 100
    issue = 0.0
    t0 = time.perf_counter()
    for _ in range(n):
        a = time.perf_counter()
        r.frame()
        issue += time.perf_counter() - a
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    print(f"{W}x{H} K={K}: wall {wall / n * 1e3:.3f} ms/frame, host issue {issue / n * 1e3:.3f} ms/frame", flush=True)
    r.close()
gl.shutdown()
