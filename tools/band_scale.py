"""Per-row cost of one band as its height grows (launch-size efficiency of the band path): the middle rank of
3 with bounds (0, c - h/2, c + h/2, H), halo exchanges stubbed. usage: python tools/band_scale.py [centre]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tools"))
sys.argv = [sys.argv[0], "3"] + sys.argv[1:2]
import band_sim as B  # noqa: E402  (sets up the GPU, scene and the stubbed exchanges; N = 3)

c = 1080
for h in [int(v) for v in os.environ.get("BAND_H", "72 144 288 576 1152 1728").split()]:
    bounds = (0, c - h // 2, c + h // 2, B.H)
    s = B.sim_rank(1, bounds)
    pp = s["pp"]
    print(f"h={h:5d} rows {s['y0']}..{s['y1']}: gbuf {pp['gbuffer']:.3f} pt {pp['pathtrace']:.3f} ms -> "
          f"per 100 rows gbuf {pp['gbuffer'] / h * 100:.3f} pt {pp['pathtrace'] / h * 100:.3f}")
