"""Dynamic scenes: 4K frames/s over GPU-built trees for several leaf sizes and PLOC radii (K = 4 frames in flight),
with the device build time. usage: python tools/dyn_sweep.py [leaf_n,radius ...]"""
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
r = Renderer(scene, 3840, 2160, parameter_config(), mode="fast", aspect_corrected=True, run_taa=False,
             run_output=False, frames_in_flight=4)
for leaf_n, radius in [tuple(int(v) for v in a.split(",")) for a in sys.argv[1:]] or [(8, 16), (4, 16), (4, 32), (8, 0)]:
    ms = [r.rebuild_bvh(leaf_n=leaf_n, ploc_radius=radius)[1] for _ in range(3)][-1]
    for _ in range(10):
        r.frame()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(150):
        r.frame()
    torch.cuda.synchronize()
    print(f"leaf_n {leaf_n} ploc {radius}: build {ms:.3f} ms, {150 / (time.perf_counter() - t0):.1f} fps", flush=True)
r.close()
gl.shutdown()
