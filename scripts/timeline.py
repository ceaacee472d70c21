"""Per-frame timeline of a rocprofv3 kernel trace: for the last frame, work (grid threads) in
flight per 0.25 ms bucket, to see how much of the frame runs with the GPU underfilled."""
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0].replace("void ", ""),
             int(r["Grid_Size_X"])) for r in rows)
frames, cur = [], []
for x in iv:
    cur.append(x)
    if "k_finalize" in x[2]:
        frames.append(cur); cur = []
f = frames[-1]
t0, t1 = f[0][0], max(e for _, e, _, _ in f)
B = 250_000
nb = (t1 - t0) // B + 1
for b in range(nb):
    lo, hi = t0 + b * B, t0 + (b + 1) * B
    thr, names = 0.0, {}
    for s, e, n, g in f:
        ov = min(e, hi) - max(s, lo)
        if ov > 0:
            w = g * ov / (e - s)
            thr += g * ov / B
            k = n.split("::")[-1].split("<")[0]
            names[k] = names.get(k, 0) + ov / B
    top = " ".join(f"{k}:{v:.2f}" for k, v in sorted(names.items(), key=lambda z: -z[1])[:4])
    print(f"{b * 0.25:6.2f} ms  avg threads {thr / 1e6:7.2f}M  {top}")
