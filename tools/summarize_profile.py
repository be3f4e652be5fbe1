"""Summarise a tools/gpu_profile.sh run into profiles/<tag>/.

* kernel_stats.csv        — rocprofv3 --kernel-trace --stats summary (copied)
* pmc_per_dispatch_avg.json — every PMC counter averaged per dispatch, per kernel
* atrous_traffic_<view>.json — HBM bytes per a-trous launch for bench.py's roofline.traffic on that camera
  view: FETCH_SIZE x 2 (gfx950 tallies 128-B streaming requests at 64 B; MI355X_MICROARCH.md
  "HBM / rocprofv3") + WRITE_SIZE, both in KiB, averaged over the LAST `REPLAY` (100) dispatches of the tile kernel:
  the launches bench.py's Renderer.time_atrous times (20 replays of the frame's 5 unfused iterations after one warm
  replay), so the bytes belong to exactly the launches whose average duration is `roofline.achieved`'s denominator
  (the frames' own launches include the fused modulate's extra bytes in one of five). It also records the a-trous
  machine code's hash (gpu_profile.sh writes it on the box: tools/kernel_hash.py), which bench.py compares with the
  library it loads: a profile of other code is reported as stale (traffic null), never as this library's.
  bench.py reads profiles/atrous_traffic_<view>.json; copy the file there from the round's directory.

usage: python tools/summarize_profile.py gpurun_out/prof_<tag> profiles/<tag> <pixels per launch> [view]
"""
import csv
import json
import os
import shutil
import sys
from collections import defaultdict

ATROUS = "atrous_tile_kernel"
REPLAY = 100  # Renderer.time_atrous(20) x 5 iterations: the timed launches, last in the bench run


def short(name: str) -> str:
    name = name.replace("void ", "")
    return name.split("(")[0]


def main(src: str, dst: str, pixels: int, view: str = "default") -> None:
    os.makedirs(dst, exist_ok=True)
    stats = os.path.join(src, "trace", "run_kernel_stats.csv")
    if os.path.exists(stats):
        shutil.copy(stats, os.path.join(dst, "kernel_stats.csv"))
    acc = defaultdict(lambda: defaultdict(list))
    replay = defaultdict(list)  # counter -> a-trous tile kernel values in dispatch order (every instantiation)
    for sub in ("fetch", "write", "sq", "l2", "sq2", "ta"):
        path = os.path.join(src, sub, "run_counter_collection.csv")
        if not os.path.exists(path):
            continue
        per = defaultdict(float)  # (kernel, counter, dispatch) -> summed value over agents/SEs
        with open(path) as f:
            for row in csv.DictReader(f):
                per[(short(row["Kernel_Name"]), row["Counter_Name"], int(row["Dispatch_Id"]))] += float(row["Counter_Value"])
        for (k, c, d), v in sorted(per.items(), key=lambda kv: kv[0][2]):  # dispatch order
            acc[k][c].append(v)
            if ATROUS in k:
                replay[c].append(v)
    avg = {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in acc.items()}
    with open(os.path.join(dst, "pmc_per_dispatch_avg.json"), "w") as f:
        json.dump(avg, f, indent=1, sort_keys=True)
    # every instantiation of the tile kernel (steps 1..16) counts as one a-trous launch; the timed replay's are last
    fetch = replay.get("FETCH_SIZE", [])[-REPLAY:]
    write = replay.get("WRITE_SIZE", [])[-REPLAY:]
    code = None
    cpath = os.path.join(src, "atrous_code_sha256.txt")
    if os.path.exists(cpath):
        with open(cpath) as f:
            code = f.read().strip() or None
    if fetch and write:
        fb = 2.0 * sum(fetch) / len(fetch) * 1024.0
        wb = sum(write) / len(write) * 1024.0
        out = {"kernel": ATROUS, "view": view, "pixels": pixels, "bytes_per_launch": round(fb + wb),
               "fetch_bytes": round(fb), "write_bytes": round(wb), "algorithmic_bytes": 52 * pixels,
               "dispatches": len(fetch), "source": os.path.basename(os.path.normpath(src)),
               "code_sha256": code,
               "method": f"FETCH_SIZE*2 + WRITE_SIZE (KiB), separate --pmc passes, the last {REPLAY} tile-kernel "
                         "dispatches (bench.py's timed a-trous replay)"}
        with open(os.path.join(dst, f"atrous_traffic_{view}.json"), "w") as f:
            json.dump(out, f, indent=1)
        print(json.dumps(out))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], int(sys.argv[3]), sys.argv[4] if len(sys.argv) > 4 else "default")
