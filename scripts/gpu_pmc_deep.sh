#!/bin/bash
# Three PMC passes (kernel-trace only) over one bench frame: instruction mix, stall split,
# cache behaviour of the traversal kernels.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-deep}
D=gpurun_out/pmc_$TAG
mkdir -p $D
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU" \
           "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INST_LEVEL_VMEM SQ_INSTS_VALU_TRANS_F32 SQ_ACTIVE_INST_SCA SQ_BUSY_CYCLES" \
           "TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE" \
           "TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TOTAL_CACHE_ACCESSES_sum" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set --kernel-trace -d $D/p$i -o p$i --output-format csv -- \
      python3 scripts/frame.py 1 > $D/p$i.out 2> $D/p$i.err || { echo "pass $i failed"; tail -5 $D/p$i.err; exit 1; }
done
python3 scripts/pmc_summary.py $D
