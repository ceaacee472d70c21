"""GPU busy/idle analysis of a rocprofv3 kernel trace: union of kernel intervals per frame."""
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
# frames: split at k_finalize
frames, cur = [], []
for s, e, n in iv:
    cur.append((s, e, n))
    if "k_finalize" in n:
        frames.append(cur); cur = []
for i, f in enumerate(frames):
    t0, t1 = f[0][0], max(e for _, e, _ in f)
    busy, end = 0, t0
    for s, e, _ in f:
        if e <= end: continue
        busy += e - max(s, end); end = e
    print(f"frame {i}: span {(t1 - t0) / 1e6:.2f} ms, busy {busy / 1e6:.2f} ms, idle {(t1 - t0 - busy) / 1e6:.2f} ms, kernels {len(f)}")
