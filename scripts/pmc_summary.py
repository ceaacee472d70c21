"""Aggregate rocprofv3 counter CSVs per kernel (sum over dispatches)."""
import collections
import csv
import glob
import sys

d = sys.argv[1]
agg = collections.defaultdict(float)
for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")[:40]
        agg[(k, r["Counter_Name"])] += float(r["Counter_Value"])
kern = sorted({k for k, _ in agg})
for k in kern:
    if not any(s in k for s in ("trace", "shadow", "shade")):
        continue
    print(k)
    for (kk, c), v in sorted(agg.items()):
        if kk == k:
            print(f"   {c:32s} {v:.4g}")
