#!/bin/bash
# SQ counters for the traversal kernels (one PMC pass, kernel-trace only).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-sq}
mkdir -p gpurun_out/pmc_$TAG
timeout -k 10 600 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --kernel-trace -d gpurun_out/pmc_$TAG/a -o a --output-format csv -- \
    python3 bench.py --steps 1 --warmup 0 --no-cpu > /dev/null 2> gpurun_out/pmc_$TAG/a.err || exit $?
timeout -k 10 600 rocprofv3 --pmc SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM_RD SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace -d gpurun_out/pmc_$TAG/b -o b --output-format csv -- \
    python3 bench.py --steps 1 --warmup 0 --no-cpu > /dev/null 2> gpurun_out/pmc_$TAG/b.err || exit $?
echo done
