"""One line per bench / probe output of a gpu_r4.sh call: ms/frame and the streams=1 kernel split.
usage: python scripts/ab_summary.py gpurun_out/<tag>"""
import json
import os
import sys

d = sys.argv[1]
for f in sorted(os.listdir(d)):
    if not f.endswith(".out"):
        continue
    for line in open(os.path.join(d, f)):
        line = line.strip()
        if line.startswith("{") and "ms_per_step" in line:
            j = json.loads(line)
            k = j.get("kernel_ms_rank0_streams1") or {}
            ks = " ".join(f"{a} {b:.2f}" for a, b in k.items())
            print(f"{f[:-4]:40s} {j['ms_per_step']:8.2f} ms  {ks}  launches {j['roofline'].get('launches')}")
        elif "render_ms" in line or line.startswith("{\"create\""):
            print(f"{f[:-4]:40s} {line}")
        elif " passed" in line or " failed" in line:
            print(f"{f[:-4]:40s} {line}")
