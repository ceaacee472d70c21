#!/bin/bash
# Per-kernel VGPR / scratch summary of the device code (cross-compiled, no GPU needed).
cd "$(dirname "$0")/../raytracer-795_amd/csrc"
hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fhip-fp32-correctly-rounded-divide-sqrt \
  -fno-gpu-flush-denormals-to-zero $EXTRA -Xclang -target-feature -Xclang -packed-fp32-ops --cuda-device-only -c rtg_device.hip -o /tmp/rtg_dev_regs.o \
  -Rpass-analysis=kernel-resource-usage 2>&1 | python3 -c '
import re, sys
name = None
for l in sys.stdin:
    m = re.search(r"Function Name: (\S+)", l)
    if m: name = m.group(1); continue
    m = re.search(r"(VGPRs|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]): (\d+)", l)
    if m and name: print(f"{name[:60]:60s} {m.group(1).split()[0]:10s} {m.group(2)}")
' | grep -E "VGPRs|Scratch|Occupancy"
