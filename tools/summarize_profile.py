"""Summarise a tools/gpu_profile.sh run into profiles/<tag>/.

* kernel_stats.csv        — rocprofv3 --kernel-trace --stats summary (copied)
* pmc_per_dispatch_avg.json — every PMC counter averaged per dispatch, per kernel
* atrous_traffic_<view>.json — HBM bytes per a-trous launch for bench.py's roofline.traffic on that camera
  view: FETCH_SIZE x 2 (gfx950 tallies 128-B streaming requests at 64 B; MI355X_MICROARCH.md
  "HBM / rocprofv3") + WRITE_SIZE, both in KiB, averaged over the tile kernel's dispatches.
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


def short(name: str) -> str:
    name = name.replace("void ", "")
    return name.split("(")[0]


def main(src: str, dst: str, pixels: int, view: str = "default") -> None:
    os.makedirs(dst, exist_ok=True)
    stats = os.path.join(src, "trace", "run_kernel_stats.csv")
    if os.path.exists(stats):
        shutil.copy(stats, os.path.join(dst, "kernel_stats.csv"))
    acc = defaultdict(lambda: defaultdict(list))
    for sub in ("fetch", "write", "sq", "l2", "sq2"):
        path = os.path.join(src, sub, "run_counter_collection.csv")
        if not os.path.exists(path):
            continue
        per = defaultdict(float)  # (kernel, counter, dispatch) -> summed value over agents/SEs
        with open(path) as f:
            for row in csv.DictReader(f):
                per[(short(row["Kernel_Name"]), row["Counter_Name"], row["Dispatch_Id"])] += float(row["Counter_Value"])
        for (k, c, _), v in per.items():
            acc[k][c].append(v)
    avg = {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in acc.items()}
    with open(os.path.join(dst, "pmc_per_dispatch_avg.json"), "w") as f:
        json.dump(avg, f, indent=1, sort_keys=True)
    # every instantiation of the step kernel (steps 1..16) counts as one a-trous launch
    fetch = [v for k, cs in acc.items() if ATROUS in k for v in cs.get("FETCH_SIZE", [])]
    write = [v for k, cs in acc.items() if ATROUS in k for v in cs.get("WRITE_SIZE", [])]
    if fetch and write:
        fb = 2.0 * sum(fetch) / len(fetch) * 1024.0
        wb = sum(write) / len(write) * 1024.0
        out = {"kernel": ATROUS, "view": view, "pixels": pixels, "bytes_per_launch": round(fb + wb),
               "fetch_bytes": round(fb), "write_bytes": round(wb), "algorithmic_bytes": 52 * pixels,
               "dispatches": len(fetch), "source": os.path.basename(os.path.normpath(src)),
               "method": "FETCH_SIZE*2 + WRITE_SIZE (KiB), separate --pmc passes"}
        with open(os.path.join(dst, f"atrous_traffic_{view}.json"), "w") as f:
            json.dump(out, f, indent=1)
        print(json.dumps(out))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], int(sys.argv[3]), sys.argv[4] if len(sys.argv) > 4 else "default")
