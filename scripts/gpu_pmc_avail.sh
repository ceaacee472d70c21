#!/bin/bash
# The texture-address / texture-data / vL1D counters this box offers (names for a TA/TD/TCP pass).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -s KILL 120 rocprofv3 --list-avail > gpurun_out/pmc_avail_full.txt 2>&1 || true
grep -E "^\s*(TA_|TD_|TCP_|SQ_INSTS_VMEM|SQ_INST_LEVEL|SQ_IFETCH|SQC_)" gpurun_out/pmc_avail_full.txt > gpurun_out/pmc_avail.txt || true
grep -oE "\b(TA|TD|TCP)_[A-Z0-9_]+" gpurun_out/pmc_avail_full.txt | sort -u > gpurun_out/pmc_avail_names.txt || true
wc -l gpurun_out/pmc_avail_full.txt gpurun_out/pmc_avail_names.txt
head -c 200000 gpurun_out/pmc_avail_full.txt > gpurun_out/pmc_avail_head.txt; rm -f gpurun_out/pmc_avail_full.txt
