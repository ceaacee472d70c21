"""Markdown rows for BASELINE.md §3 / README from bench lines (one JSON line per file).

usage: python scripts/baseline_table.py <bench.json> ...   (e.g. profiles/history/r3d_bench_final_*.json)
Columns: workload, spp, ms/frame, Mray/s, primary Msamples/s, ms/frame incl. D2H, scene create ms,
first frame incl. D2H ms, frame HBM GB/s (frac of 8 TB/s), parity (oracle rows, differing values).
"""
import json
import sys


def row(d):
    c = d["config"]
    r = d.get("roofline") or {}
    fh = r.get("frame_hbm")
    hbm = f"{fh['achieved']:,.0f} ({fh['frac']:.2f})" if fh else "—"
    p = d.get("parity")
    par = f"rows {p['rows'][0]}–{p['rows'][1]}: {p['differing']} differing" if p else "—"
    e = d["end_to_end_ms"]
    name = c["workload"].split(":")[0]
    again = e.get("scene_create_again")
    create = f"{e['scene_create']:.0f}" + (f" / {again['ms']:.0f}" if again else "")
    return (f"| {name} | {c['spp']} | {d['ms_per_step']:.2f} | {d['value']:,.0f} | {d['primary_msamples_s']:,.0f} | "
            f"{d['ms_per_frame_to_host']:.2f} | {create} | {e['first_frame_to_host']:.0f} | {hbm} | {par} |")


def main():
    print("| config (workload) | spp | ms/frame | Mray/s | primary Msamples/s | ms/frame incl. D2H | scene create ms (first / again) "
          "| first frame incl. D2H ms | frame HBM GB/s (frac of 8 TB/s) | parity vs oracle |")
    print("|---|---|---|---|---|---|---|---|---|---|")
    for f in sys.argv[1:]:
        with open(f) as fh:
            line = [x for x in fh.read().splitlines() if x.startswith("{")][-1]
        print(row(json.loads(line)))


if __name__ == "__main__":
    main()
