#!/bin/bash
# VGPR / SGPR / spill / scratch of the traversal and shading kernels in a gfx950 build of rtg_device.hip
# (dev tool: cross-compiles the device code to assembly and reads its kernel metadata).
#   bash scripts/regs_report.sh [extra hipcc flags]
set -e
cd "$(dirname "$0")/../raytracer-795_amd/csrc"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fhip-fp32-correctly-rounded-divide-sqrt \
  -fno-gpu-flush-denormals-to-zero -Xclang -target-feature -Xclang -packed-fp32-ops --offload-device-only -S \
  -o /tmp/rtg_dev.s rtg_device.hip "$@" 2>&1 | grep -v "not a recognized\|hip-link" || true
python3 - <<'PY'
import re
s = open('/tmp/rtg_dev.s').read()
for m in re.finditer(r'\.name:\s+(\S+)\n(.*?)\.vgpr_count:\s+(\d+)', s, re.S):
    pass
# amdhsa metadata blocks: one per kernel
for blk in s.split('  - .agpr_count')[1:]:
    name = re.search(r'\.name:\s+(\S+)', blk).group(1)
    if not re.search(r'k_(trace|shadow|shade|pt_shade)', name):
        continue
    g = lambda k: (re.search(r'\.' + k + r':\s+(\d+)', blk) or [0, '?'])[1]
    dem = name.replace('_ZN3rtg', '')[:60]
    print(f"{dem:60s} vgpr {g('vgpr_count'):>4} sgpr {g('sgpr_count'):>4} vspill {g('vgpr_spill_count'):>4} "
          f"sspill {g('sgpr_spill_count'):>4} scratch {g('private_segment_fixed_size'):>5}")
PY
