"""Per-wave timeline of wf_primary (investigation build -DPT_WAVE_TIMES): each wave's start/end (s_memrealtime,
100 MHz) and its largest traversal step count, for the full 4K frame and for a thin band. Shows how long the
launch's tail is and the latency per traversal step of the slowest waves.
usage: PTSVGF_LIB_DIR=.../lib_exp/wavetimes python tools/archive/wave_times.py
Archived in round 4: the PT_WAVE_TIMES blocks left kernels_wavefront.hip (they are at commit d4ff747); rebuild that
revision's library with -DPT_WAVE_TIMES to use this script."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "path-tracing-svgf_amd"))
sys.path.insert(0, os.path.join(REPO, "tools"))
import numpy as np
import torch

import band_sim as B  # noqa: E402  (GPU, scene, stubbed exchanges)
from ptsvgf import dist as D


def run(bounds, tag):
    r = D.BandRenderer(B.scene, B.W, B.H, B.cfg, 1, 3, B.FakeDist(), bounds=bounds)
    for _ in range(2):
        r.frame()
    n = (B.W // 16 + 1) * ((r.plan.y1 - r.plan.y0) // 16 + 1) * 4 * 4
    c = torch.zeros(n, dtype=torch.int32, device="cuda")
    r.pass_path_tracing.set_row_cost(c.data_ptr())
    r.frame()
    torch.cuda.synchronize()
    r.pass_path_tracing.set_row_cost(0)
    a = c.cpu().numpy().view(np.uint32).reshape(-1, 4)
    a = a[a[:, 3] == 1].astype(np.int64)
    t0 = a[:, 0].min()
    st, en, steps = (a[:, 0] - t0) / 100.0, (a[:, 1] - t0) / 100.0, a[:, 2]  # microseconds
    dur = en - st
    end = en.max()
    print(f"--- {tag}: rows {r.plan.y0}..{r.plan.y1}, {len(a)} waves, launch span {end:.1f} us")
    for q in (50, 90, 99, 100):
        print(f"  wave end time p{q}: {np.percentile(en, q):.1f} us;  wave duration p{q}: {np.percentile(dur, q):.1f} us")
    k = np.argsort(dur)[::-1][:8]
    for i in k:
        print(f"  slow wave: start {st[i]:.1f} end {en[i]:.1f} dur {dur[i]:.1f} us, max steps {steps[i]}, "
              f"{dur[i] / max(steps[i], 1) * 1e3:.0f} ns/step")
    sel = steps > 200
    if sel.any():
        print(f"  waves with >200 steps: median ns/step {np.median(dur[sel] / steps[sel]) * 1e3:.0f}")
    r.close()


run(None, "equal thirds, middle band")
run((0, 1044, 1116, B.H), "72-row band")
run((0, 36, 2124, B.H), "nearly full frame")
