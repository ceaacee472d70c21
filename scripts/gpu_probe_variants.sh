#!/bin/bash
# Probe (stats + timing) for the default library and each dev variant in $VARIANTS.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in librtg.so $VARIANTS; do
  echo "== variant $v"
  RTG_LIBRARY=raytracer-795_amd/rtg/$v timeout -k 10 300 python scripts/probe.py ${1:-dragon1m} ${2:-64} > gpurun_out/probe_$v.log 2>&1 || { cat gpurun_out/probe_$v.log; exit 1; }
  cat gpurun_out/probe_$v.log
done
