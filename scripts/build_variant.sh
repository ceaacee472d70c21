#!/bin/bash
# Dev variants of librtg.so for A/B timing on the GPU box:
#   scripts/build_variant.sh <name> [extra hipcc flags...]  ->  raytracer-795_amd/rtg/<name>.so
# Run them with VARIANTS="<name>.so ..." scripts/gpu_quick.sh (RTG_LIBRARY selects the library).
set -e
cd "$(dirname "$0")/../raytracer-795_amd/csrc"
name=$1; shift
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -shared -std=c++17 -ffp-contract=off \
  -fhip-fp32-correctly-rounded-divide-sqrt -fno-gpu-flush-denormals-to-zero -Wno-unused-result \
  "$@" -o ../rtg/$name.so rtg_device.hip rtg_host.cpp
