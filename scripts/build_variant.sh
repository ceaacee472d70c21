#!/bin/bash
# Dev variants of librtg.so for A/B timing on the GPU box:
#   scripts/build_variant.sh <name> [extra hipcc flags...]  ->  raytracer-795_amd/rtg/<name>.so
# Run them with CONFIGS="<name>:<streams> ..." scripts/gpu_ab.sh (RTG_LIBRARY selects the library).
set -e
cd "$(dirname "$0")/../raytracer-795_amd/csrc"
name=$1; shift
make -s OUT=../rtg/$name.so OBJ=../../build/variant_$name EXTRA="$*"
