#!/bin/bash
# kernel timeline of one simulated band (rank 4 of 8, equal bands, K frames in flight) + GPU busy fraction
R="$GRAFT_REPO_ROOT"
cd /tmp && export TMPDIR=/tmp
export GPU_MAX_HW_QUEUES=16 BALANCE=0 RANKS=4 FIF=${FIF:-4}
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/bt" -o run -- python3 "$R/tools/band_sim.py" 8 > "$R/gpurun_out/bt.log" 2>&1 || exit $?
python3 - "$R/gpurun_out/bt/run_kernel_trace.csv" <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
# last 40% of the run (steady state frames)
t0, t1 = ev[0][0], max(e[1] for e in ev)
lo = t0 + 0.6 * (t1 - t0)
ev = [e for e in ev if e[0] >= lo]
# union of busy intervals
busy, cur_s, cur_e = 0, None, None
for s, e, _ in ev:
    if cur_e is None or s > cur_e:
        if cur_e is not None: busy += cur_e - cur_s
        cur_s, cur_e = s, e
    else:
        cur_e = max(cur_e, e)
busy += cur_e - cur_s
span = max(e[1] for e in ev) - ev[0][0]
print(f"window {span/1e6:.2f} ms, GPU busy (any kernel running) {busy/span*100:.1f}%")
tot = collections.defaultdict(float); cnt = collections.Counter()
for s, e, n in ev:
    k = n.split("(")[0].replace("void ", "")[:40]; tot[k] += (e - s) / 1e6; cnt[k] += 1
for k, v in sorted(tot.items(), key=lambda x: -x[1])[:14]:
    print(f"  {k:40s} n={cnt[k]:4d} sum {v:7.2f} ms avg {v/cnt[k]*1e3:7.1f} us")
PY
