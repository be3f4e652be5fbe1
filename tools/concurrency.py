"""How full the GPU is inside bench.py's timed region, from a rocprofv3 kernel trace.

The timed region is the span between the two `torch.arange` marker kernels bench.py launches right before and right
after its timed loop. Prints: the region's length per frame, the share of that time with 0, 1, 2, ... kernels
resident, the kernels that run alone (and the most common pairs), and each kernel's summed duration per frame (a
kernel's duration counts all the time it shares the GPU with others, so these sums exceed the frame).
usage: python tools/concurrency.py gpurun_out/prof_<tag>/trace/run_kernel_trace.csv [frames=5]"""
import csv
import sys


def short(name: str) -> str:
    return name.split("(")[0].replace("void ", "")[:60]


def main(path: str, frames: int) -> None:
    rows = list(csv.DictReader(open(path)))
    raw = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
    marks = [(s, e) for s, e, n in raw if "arange" in n]
    if len(marks) < 2:
        sys.exit("no pair of arange marker kernels in the trace (bench.py's timed-region markers)")
    w0, w1 = marks[0][1], marks[1][0]
    ks = [(max(s, w0), min(e, w1), short(n)) for s, e, n in raw if min(e, w1) > max(s, w0)]
    pts = sorted({s for s, _, _ in ks} | {e for _, e, _ in ks} | {w0, w1})
    hist, alone, pair, summed = {}, {}, {}, {}
    for s, e, n in ks:
        summed[n] = summed.get(n, 0) + (e - s)
    for a, b in zip(pts, pts[1:]):
        act = [n for s, e, n in ks if s <= a and e >= b]
        hist[len(act)] = hist.get(len(act), 0) + (b - a)
        if len(act) == 1:
            alone[act[0]] = alone.get(act[0], 0) + (b - a)
        elif len(act) == 2:
            k = " + ".join(sorted(act))
            pair[k] = pair.get(k, 0) + (b - a)
    span = w1 - w0
    print(f"timed region: {span / 1e6:.3f} ms = {span / 1e6 / frames:.3f} ms per frame ({frames} frames)")
    print("kernels resident: share of the region")
    for k in sorted(hist):
        print(f"  {k}: {hist[k] / span:.3f}")
    print("running alone, ms per frame:")
    for n, v in sorted(alone.items(), key=lambda x: -x[1])[:10]:
        print(f"  {v / 1e6 / frames:.3f}  {n}")
    print("two kernels together, ms per frame:")
    for n, v in sorted(pair.items(), key=lambda x: -x[1])[:8]:
        print(f"  {v / 1e6 / frames:.3f}  {n}")
    print("summed kernel durations, ms per frame (overlapping):")
    for n, v in sorted(summed.items(), key=lambda x: -x[1])[:16]:
        print(f"  {v / 1e6 / frames:.3f}  {n}")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 5)
