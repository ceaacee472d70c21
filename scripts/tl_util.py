"""GPU occupancy of the last frame of a rocprofv3 kernel trace (scripts/tl_probe.py):
frame span, time with no kernel running, time with fewer than `full` threads in flight, and per
kernel its launches, total and median duration and the time spent in small launches.
usage: python scripts/tl_util.py <kernel_trace.csv> [full_threads]"""
import csv
import statistics
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
full = int(sys.argv[2]) if len(sys.argv) > 2 else 256 * 4 * 64 * 2
iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
             r["Kernel_Name"].split("(")[0].replace("void ", "").split("::")[-1].split("<")[0],
             int(r["Grid_Size_X"])) for r in rows)
frames, cur = [], []
for x in iv:
    cur.append(x)
    if x[2] == "k_finalize":
        frames.append(cur)
        cur = []
f = frames[-1]
t0, t1 = f[0][0], max(e for _, e, _, _ in f)
ev = []
for s, e, n, g in f:
    ev.append((s, g))
    ev.append((e, -g))
ev.sort()
idle = under = 0
thr = 0
last = t0
for t, dg in ev:
    if t > last:
        if thr == 0:
            idle += t - last
        elif thr < full:
            under += t - last
        last = t
    thr += dg
span = t1 - t0
print(f"frame span {span / 1e6:.2f} ms, no kernel {idle / 1e6:.2f} ms, < {full} threads {under / 1e6:.2f} ms "
      f"({(idle + under) / span:.1%} of the frame underfilled)")
by = {}
for s, e, n, g in f:
    by.setdefault(n, []).append((e - s, g))
for n, v in sorted(by.items(), key=lambda z: -sum(d for d, _ in z[1])):
    d = [x for x, _ in v]
    small = sum(x for x, g in v if g < full)
    print(f"{n:16s} launches {len(v):5d}  total {sum(d) / 1e6:8.2f} ms  median {statistics.median(d) / 1e3:8.1f} us"
          f"  small-grid launches {sum(1 for _, g in v if g < full):5d} ({small / 1e6:.2f} ms)")
