"""Locate path-tracer pixels that differ from the oracle (diagnostic)."""
import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "path-tracing-svgf_amd")); sys.path.insert(0, os.path.join(REPO, "tests"))
import numpy as np
import oracle_ref as O
from ptsvgf import gl
from ptsvgf.renderer import Renderer
from ptsvgf.scene import build_scene

W = H = int(os.environ.get("DBG_RES", "64"))
scene = build_scene("table_clock_plant", hdr_size=(256, 128), plant_leaves=40)
print("nan in tri normals:", int(np.isnan(scene.tri_enc[:, 9:18]).sum()))
gl.init(0)
ref = O.OracleFrameLoop(scene, W, H)
want = ref.frame()
res = {}
for name, kern, prune in (("wavefront", 0, 1), ("mega", 1, 1), ("mega_noprune", 1, 0), ("wave_noprune", 0, 0)):
    r = Renderer(scene, W, H, mode="fast", prune=bool(prune), run_taa=False, run_output=False)
    r.pass_path_tracing.set_uniform_int("pt_kernel", kern)
    r.frame()
    got = gl.readback(r.planes()["color"])
    res[name] = got
    bad = np.argwhere(np.any(got != want["color"], axis=-1))
    print(f"{name}: {len(bad)} differing pixels; max diff {np.nanmax(np.abs(got - want['color'])):.4g}")
    for (y, x) in bad[:6]:
        print("   px", x, y, "gpu", got[y, x, :3], "oracle", want["color"][y, x, :3])
print("mega vs wave equal:", np.array_equal(res["mega"], res["wavefront"]),
      "noprune mega vs prune mega:", np.array_equal(res["mega"], res["mega_noprune"]))
gl.shutdown()
