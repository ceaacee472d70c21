"""Per-kernel PMC counters of a gpu_round.sh run -> one CSV + one JSON summary.

usage: python scripts/pmc_counters.py <prof_dir> <out.csv> <out.json> [workload]

Every counter pass (p1..pN) is a separate `rocprofv3 --pmc <set> --kernel-trace` run of
`bench.py --steps 1 --warmup 0 --no-cpu --streams 1`.  For each kernel and counter the
CSV holds the number of dispatches, the sum over them and the mean per dispatch; the JSON holds
the per-dispatch means that bench.py divides by its live HIP-event launch times (the roofline
ceilings of DESIGN.md §4).  FETCH_SIZE / WRITE_SIZE are in KB; the gfx950 correction
(MI355X_MICROARCH.md §HBM: FETCH_SIZE reports half the bytes of wide reads) is applied in the
JSON's `hbm_bytes` (= 2 x FETCH_SIZE x 1024 + WRITE_SIZE x 1024).
"""
import collections
import csv
import glob
import json
import os
import sys


def kname(k):
    # the scene-build and tone-map kernels live in anonymous namespaces (rtg::anon::k_*); the frame's
    # kernels (rtg_device.hip) in rtg:: itself
    k = k.replace("(anonymous namespace)::", "anon::").split("(")[0].replace("void ", "")
    return k


# Kernels whose level-0 and queued-level instantiations (last template argument) bench.py times
# together: one combined entry each as well, `<prefix>, *>` (e.g. k_trace<false, false, *>).
COMBINED = ("rtg::k_trace<false, false", "rtg::k_shadow<false, false", "rtg::k_shade<false, false, 512, false", "rtg::k_shade<false, true, 512, false",
            "rtg::k_shade<true, true, 256, false", "rtg::k_shade<true, true, 256, true",
            "rtg::k_shade<true, false, 256, false", "rtg::k_shade<true, false, 256, true",
            "rtg::k_shade<true, false, 512, false",
            "rtg::k_pt_shade<false, false, true", "rtg::k_pt_shade<false, false, false", "rtg::k_pt_shade<false, true, true",
            "rtg::k_pt_shade<true, true, true", "rtg::k_pt_shade<true, false, true",
            "rtg::k_pt_shade<false, false, 0", "rtg::k_pt_shade<false, false, 1", "rtg::k_pt_shade<false, false, 2",
            "rtg::k_pt_shade<false, true, 0", "rtg::k_pt_shade<false, true, 1", "rtg::k_pt_shade<false, true, 2",
            "rtg::k_pt_shade<true, true, 2", "rtg::k_pt_shade<true, false, 2")


def keys_of(k):
    return {k} | {p + ", *>" for p in COMBINED if k.startswith(p + ",")}


def main():
    d, out_csv, out_json = sys.argv[1:4]
    workload = sys.argv[4] if len(sys.argv) > 4 else "dragon1m"
    tot = collections.defaultdict(float)
    cnt = collections.defaultdict(int)
    for f in sorted(glob.glob(f"{d}/p*/**/*counter_collection.csv", recursive=True)):
        for r in csv.DictReader(open(f)):
            k = kname(r["Kernel_Name"])
            c = r["Counter_Name"]
            v = float(r["Counter_Value"])
            for key in keys_of(k):
                tot[(key, c)] += v
                cnt[(key, c)] += 1
    rows = sorted(tot)
    with open(out_csv, "w", newline="") as fh:
        w = csv.writer(fh)
        w.writerow(["kernel", "counter", "dispatches", "sum", "per_dispatch"])
        for k, c in rows:
            w.writerow([k, c, cnt[(k, c)], f"{tot[(k, c)]:.6g}", f"{tot[(k, c)] / cnt[(k, c)]:.6g}"])
    summ = collections.defaultdict(dict)
    for k, c in rows:
        summ[k][c] = tot[(k, c)] / cnt[(k, c)]
        summ[k]["dispatches_" + c] = cnt[(k, c)]
    for k, m in summ.items():
        if "FETCH_SIZE" in m and "WRITE_SIZE" in m:
            m["hbm_bytes"] = 2.0 * m["FETCH_SIZE"] * 1024 + m["WRITE_SIZE"] * 1024
    json.dump({"source": os.path.basename(os.path.normpath(d)), "workload": workload,
               "command": "rocprofv3 --pmc <set> --kernel-trace -- python3 bench.py --steps 1 --warmup 0 --no-cpu --streams 1",
               "kernels": summ}, open(out_json, "w"), indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
