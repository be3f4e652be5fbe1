import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
# take the last 40% of the trace (steady state)
t0, t1 = iv[0][0], max(e for _, e, _ in iv)
cut = t0 + (t1 - t0) * 0.6
iv = [(max(s, cut), e, n) for s, e, n in iv if e > cut]
busy = 0; cur_s = None; cur_e = None
for s, e, _ in iv:
    if cur_e is None or s > cur_e:
        if cur_e is not None: busy += cur_e - cur_s
        cur_s, cur_e = s, e
    else:
        cur_e = max(cur_e, e)
busy += cur_e - cur_s
span = t1 - cut
print(f"window {span/1e6:.2f} ms, busy (any kernel running) {busy/span*100:.1f}%")
# concurrency histogram: average number of concurrent kernels
ev = []
for s, e, _ in iv: ev += [(s, 1), (e, -1)]
ev.sort(); c = 0; last = ev[0][0]; acc = 0
for t, d in ev:
    acc += c * (t - last); c += d; last = t
print(f"mean concurrent kernels {acc/span:.2f}")
