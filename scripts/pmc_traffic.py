"""Per-kernel HBM traffic from separate rocprofv3 `--pmc FETCH_SIZE` / `--pmc WRITE_SIZE` passes.

usage: python scripts/pmc_traffic.py <prof_dir> <out.json> [command description]

FETCH_SIZE / WRITE_SIZE are in KB.  gfx950 correction (MI355X_MICROARCH.md, HBM/rocprofv3
section): FETCH_SIZE reports half of the bytes of wide streaming reads -> read bytes =
2 x FETCH_SIZE x 1024; WRITE_SIZE is exact for 16-B-per-lane stores.  Infinity-Cache hits
may be counted by these fabric-side counters.
"""
import collections
import csv
import glob
import json
import sys


def per_kernel(d, counter):
    tot = collections.defaultdict(float)
    n = collections.defaultdict(int)
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter:
                continue
            k = r["Kernel_Name"].split("(")[0].replace("void ", "")
            tot[k] += float(r["Counter_Value"])
            n[k] += 1
    return {k: (n[k], tot[k] / n[k]) for k in tot}


def main():
    d, out = sys.argv[1], sys.argv[2]
    cmd = sys.argv[3] if len(sys.argv) > 3 else ""
    fetch = per_kernel(f"{d}/fetch", "FETCH_SIZE")
    write = per_kernel(f"{d}/write", "WRITE_SIZE")
    res = {}
    for k in sorted(set(fetch) | set(write)):
        nf, fkb = fetch.get(k, (0, 0.0))
        nw, wkb = write.get(k, (0, 0.0))
        res[k] = {"launches_fetch_pass": nf, "launches_write_pass": nw,
                  "fetch_kb_raw_per_launch": round(fkb, 1), "write_kb_per_launch": round(wkb, 1),
                  "hbm_bytes_per_launch": round(2 * fkb * 1024 + wkb * 1024)}
    # the closest-hit kernel has two instantiations on the bench path (GEN=true: level 0 of the
    # Whitted path generating its primary rays; GEN=false: secondary levels): a launch-weighted
    # combined entry is what bench.py's roofline (HIP events over all its launches) compares to
    parts = [k for k in res if k.startswith("rtg::k_trace<false, false")]
    if parts:
        nl = sum(res[k]["launches_fetch_pass"] for k in parts)
        if nl:
            res["rtg::k_trace<false, false, *>"] = {
                "launches_fetch_pass": nl, "parts": parts,
                "hbm_bytes_per_launch": round(sum(res[k]["hbm_bytes_per_launch"] * res[k]["launches_fetch_pass"]
                                                  for k in parts) / nl)}
    json.dump({"kernels": res, "command": cmd,
               "note": "hbm_bytes_per_launch = 2 x FETCH_SIZE(KB) x 1024 + WRITE_SIZE(KB) x 1024 "
                       "(gfx950 FETCH_SIZE half-count correction); averaged over the dispatches of the pass"},
              open(out, "w"), indent=1)
    for k, v in res.items():
        print(f"{k[:60]:60s} {v['hbm_bytes_per_launch'] / 1e6:10.2f} MB/launch")


if __name__ == "__main__":
    main()
