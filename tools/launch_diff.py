"""Launch-by-launch comparison of rocprofv3 kernel traces (round 6): a simulated frame-shard rank
(tools/frame_shard_sim.py under tools/shard_diff.sh) against the one-GPU bench frame at K = 1 and K = 4.

Only the timed frames count: the runs launch torch.arange(3) right before and right after their timed region, and the
kernels between those two marker launches are taken. Per trace and kernel: launches and summed duration per frame of
the run's rate, and the mean duration of one launch. Per trace: the GPU's busy time (the union of kernel intervals) and
the summed kernel time per frame (their ratio = mean kernels running at once).

A simulated rank draws every frame's band work (G-buffer on its ghost-zone rows, SVGF chain) and every N-th frame's
whole-frame G-buffer + path tracer; its per-frame path-tracer figures are therefore compared per OWN frame (x N).

usage: python tools/launch_diff.py TRACE_DIR:FRAMES[:OWN_EVERY] ... (a label = the directory's basename)"""
import csv
import glob
import os
import re
import sys

PT = ("wf_", "pr_", "tile_sort", "primary", "hdr_merge")
GBUF = ("gbuffer", "rast_", "bins_", "atrous_flags", "gbuf")
SVGF = ("reproject", "variance", "atrous", "modulate", "taa")


def short(name: str) -> str:
    n = re.sub(r"^void ", "", name)
    n = re.sub(r"\(.*$", "", n)  # argument list
    n = n.replace("ptk::", "")
    return n[:90]


def family(name: str, grid: int, full_grid: int) -> str:
    n = name
    if "arange" in n:
        return "marker"
    if any(k in n for k in PT):
        return "path tracer"
    if any(k in n for k in GBUF):
        return "G-buffer (whole frame)" if grid >= full_grid else "G-buffer (band)"
    if any(k in n for k in SVGF):
        return "SVGF"
    if "sleep" in n.lower() or "spin" in n.lower():
        return "comm stand-in"
    return "copies / other"


def load(path: str):
    f = path if path.endswith(".csv") else (glob.glob(os.path.join(path, "**", "*kernel_trace.csv"), recursive=True)
                                            or [None])[0]
    if f is None:
        raise FileNotFoundError(f"no kernel_trace.csv under {path}")
    rows = []
    with open(f) as fh:
        for r in csv.DictReader(fh):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"],
                         int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"]), int(r["Queue_Id"])))
    rows.sort()
    marks = [i for i, r in enumerate(rows) if "arange" in r[2] or "elementwise_kernel_with_index" in r[2]]
    if len(marks) >= 2:
        t0, t1 = rows[marks[-2]][1], rows[marks[-1]][0]
        rows = [r for r in rows if r[0] >= t0 and r[1] <= t1]
    else:
        t0, t1 = rows[0][0], rows[-1][1]
        print(f"  ({path}: no timed-region markers; whole trace)")
    return rows, t0, t1


def union(iv):
    tot, cur0, cur1 = 0, None, None
    for a, b in sorted(iv):
        if cur1 is None or a > cur1:
            if cur1 is not None:
                tot += cur1 - cur0
            cur0, cur1 = a, b
        else:
            cur1 = max(cur1, b)
    return tot + ((cur1 - cur0) if cur1 is not None else 0)


def summarize(path: str, frames: int, own_every: int):
    rows, t0, t1 = load(path)
    full_grid = max((g for _, _, n, g, _ in rows if any(k in n for k in GBUF)), default=0)
    per = {}
    fam = {}
    for a, b, n, g, q in rows:
        k = short(n)
        d = (b - a) / 1e3  # us
        e = per.setdefault(k, [0, 0.0])
        e[0] += 1
        e[1] += d
        fk = family(n, g, full_grid)
        fam[fk] = fam.get(fk, 0.0) + d
    # the SVGF chain of each frame (reproject, variance, five a-trous launches on one stream): its span from the
    # reprojection's start to the last a-trous launch's end, against its kernels' summed time (the rest is waiting for
    # CUs held by other streams' kernels, or for the chain's own inputs)
    chains = []
    svgf = [(a, b, n, q) for a, b, n, g, q in rows if any(k in n for k in SVGF)]
    for i, (a, b, n, q) in enumerate(svgf):
        if "reproject" not in n:
            continue
        same = [x for x in svgf[i:] if x[3] == q]
        at = [x for x in same if "atrous" in x[2]][:5]
        if len(at) == 5:
            span = at[-1][1] - a
            busy_k = sum(x[1] - x[0] for x in same if x[0] <= at[-1][0])
            chains.append((span / 1e3, busy_k / 1e3))
    wall = (t1 - t0) / 1e3 / frames
    busy = union([(a, b) for a, b, *_ in rows]) / 1e3 / frames
    ksum = sum(d for _, d in per.values()) / frames
    print(f"== {os.path.basename(path.rstrip('/'))}: {frames} frames, {wall / 1e3:.3f} ms/frame wall, GPU busy "
          f"{busy / 1e3:.3f} ms/frame ({busy / wall:.0%}), kernel time {ksum / 1e3:.3f} ms/frame "
          f"({ksum / max(busy, 1e-9):.2f} kernels at once)")
    if chains:
        import statistics
        print(f"   SVGF chain per frame: span {statistics.median(c[0] for c in chains) / 1e3:.3f} ms median "
              f"(p90 {sorted(c[0] for c in chains)[int(0.9 * (len(chains) - 1))] / 1e3:.3f}), its kernels "
              f"{statistics.median(c[1] for c in chains) / 1e3:.3f} ms ({len(chains)} chains)")
    for fk, d in sorted(fam.items(), key=lambda x: -x[1]):
        per_own = f" = {d / frames * own_every / 1e3:.3f} ms per own frame" if own_every > 1 and fk in (
            "path tracer", "G-buffer (whole frame)") else ""
        print(f"   {fk:24s} {d / frames / 1e3:.3f} ms/frame{per_own}")
    return per, frames, own_every, wall


def main():
    runs = []
    for arg in sys.argv[1:]:
        parts = arg.split(":")
        path, frames = parts[0], int(parts[1])
        own = int(parts[2]) if len(parts) > 2 else 1
        runs.append((os.path.basename(path.rstrip("/")), summarize(path, frames, own)))
    names = sorted({k for _, (per, *_r) in runs for k in per if any(p in k for p in PT + GBUF)},
                   key=lambda k: -max(per.get(k, [0, 0.0])[1] / fr * own for _, (per, fr, own, _w) in runs))
    print("\npath-tracer and G-buffer launches, per traced frame (a simulated rank: per own frame): launches, "
          "summed us, mean us per launch")
    hdr = "kernel".ljust(60) + "".join(f"{lab[:26]:>30s}" for lab, _ in runs)
    print(hdr)
    for k in names:
        line = k[:59].ljust(60)
        for _, (per, fr, own, _w) in runs:
            c, d = per.get(k, [0, 0.0])
            if c:
                line += f"{c / fr * own:8.1f} {d / fr * own:10.1f} {d / c:9.1f}  "
            else:
                line += " " * 30
        print(line)


if __name__ == "__main__":
    main()
