"""Markdown per-kernel roofline table from one bench line's `roofline.kernels`.

usage: python scripts/roofline_table.py profiles/history/r3f_<workload>_bench_final.json
Columns: kernel, ms / frame (streams=1 roofline frame), launches, VALU frac (lane-adjusted), HBM GB/s
(frac of 8 TB/s), HBM MB / launch, L2 hit, issuing / waiting on memory / dependency, lane efficiency.
"""
import json
import sys


def main():
    with open(sys.argv[1]) as fh:
        d = json.loads([x for x in fh.read().splitlines() if x.startswith("{")][-1])
    ks = d["roofline"]["kernels"]
    print("| kernel | ms / frame | launches | VALU frac (lane-adj.) | HBM GB/s (frac) | HBM MB / launch | L2 hit "
          "| issuing / mem wait / dep. | lane eff. |")
    print("|---|---|---|---|---|---|---|---|---|")
    for name, k in ks.items():
        v, h, w = k.get("valu", {}), k.get("hbm", {}), k.get("wave_cycles", {})
        adj = v.get("lane_adjusted_frac")
        vf = f"{v.get('frac', 0):.2f}" + (f" ({adj:.2f})" if adj is not None else "")
        ms = k["avg_launch_ms"] * k["launches"]
        eff = k.get("simd_eff")
        print(f"| `{name}` | {ms:.2f} | {k['launches']} | {vf} | {h.get('achieved', 0):,.0f} ({h.get('frac', 0):.2f}) | "
              f"{h.get('bytes_per_launch', 0) / 1e6:,.0f} | {k.get('l2_hit_rate', 0):.2f} | "
              f"{w.get('issuing', 0):.2f} / {w.get('waiting_on_memory', 0):.2f} / {w.get('issue_stalled', 0):.2f} | "
              f"{'' if eff is None else f'{eff:.2f}'} |")
    fh = d["roofline"].get("frame_hbm")
    if fh:
        print(f"\nframe: {d['ms_per_step']:.2f} ms, HBM {fh['achieved']:,.0f} GB/s ({fh['frac']:.2f} of 8 TB/s)")


if __name__ == "__main__":
    main()
