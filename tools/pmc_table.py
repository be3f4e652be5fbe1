"""Per-kernel PMC metrics from a summarize_profile.py output directory, as a markdown table.

VALU busy = SQ_INSTS_VALU x 2 cycles (a wave64 VALU instruction issues over 2 cycles on a SIMD-32,
MI355X_MICROARCH.md "Wave scheduling") / (1024 SIMDs x GRBM_GUI_ACTIVE / 8 cycles: the counter sums the 8 XCDs);
waiting = SQ_WAIT_ANY / SQ_WAVE_CYCLES (waves parked on s_waitcnt / barriers), issue-stalled = SQ_WAIT_INST_ANY /
SQ_WAVE_CYCLES, L2 hit = TCC_HIT / (TCC_HIT + TCC_MISS). PMC passes serialise dispatches, so these describe each
kernel alone; the duration column is the kernel trace's average of the same run configuration.

usage: python tools/pmc_table.py profiles/r03/k4_default [kernel substrings...]
"""
import csv
import json
import os
import sys


def short(name: str) -> str:
    return name.replace("void ", "").split("(")[0]


def main(d, keys):
    pmc = json.load(open(os.path.join(d, "pmc_per_dispatch_avg.json")))
    dur = {}
    ks = os.path.join(d, "kernel_stats.csv")
    if os.path.exists(ks):
        for row in csv.DictReader(open(ks)):
            dur[short(row["Name"])] = (int(row["Calls"]), float(row["AverageNs"]) / 1e3, float(row["Percentage"]))
    print("| kernel | calls | avg µs | % GPU time | VALU busy | waiting | issue-stalled | L2 hit | VALU instr / wave |")
    print("|---|---|---|---|---|---|---|---|---|")
    for k in sorted(pmc, key=lambda k: -dur.get(k, (0, 0, 0))[2]):
        if keys and not any(s in k for s in keys):
            continue
        c = pmc[k]
        cyc = c.get("GRBM_GUI_ACTIVE", 0) / 8
        valu = c.get("SQ_INSTS_VALU", 0) * 2 / (1024 * cyc) if cyc else float("nan")
        wc = c.get("SQ_WAVE_CYCLES", 0)
        wait = c.get("SQ_WAIT_ANY", 0) / wc if wc else float("nan")
        stall = c.get("SQ_WAIT_INST_ANY", 0) / wc if wc else float("nan")
        h, m = c.get("TCC_HIT_sum", 0), c.get("TCC_MISS_sum", 0)
        hit = h / (h + m) if h + m else float("nan")
        per_wave = c.get("SQ_INSTS_VALU", 0) / c["SQ_WAVES"] if c.get("SQ_WAVES") else float("nan")
        n, us, pct = dur.get(k, (0, float("nan"), float("nan")))
        print(f"| `{k}` | {n} | {us:.1f} | {pct:.1f} | {valu:.1%} | {wait:.1%} | {stall:.1%} | {hit:.1%} | {per_wave:.0f} |")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2:])
