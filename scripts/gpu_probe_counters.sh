#!/bin/bash
# Probe (stats incl. SIMD efficiency) + list of available SQ counters on this box.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python scripts/probe.py ${1:-dragon1m} ${2:-64} > gpurun_out/probe.log 2>&1 || { cat gpurun_out/probe.log; exit 1; }
cat gpurun_out/probe.log
timeout -k 10 120 rocprofv3 --list-avail > gpurun_out/avail.txt 2>&1
grep -o "SQ_[A-Z_0-9]*" gpurun_out/avail.txt | sort -u | tr '\n' ' ' > gpurun_out/sq_counters.txt
echo; wc -c gpurun_out/sq_counters.txt
