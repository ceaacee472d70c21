#!/bin/bash
# Texture-address / texture-data / vL1D pressure of the frame kernels (is the divergent gather
# path the bound?): two PMC passes (<= 2 TA, 2 TD, 4 TCP counters each) over one bench frame
# with RTG_STREAMS=1, summarised per kernel by pmc_counters.py.
#   gpurun -- bash scripts/gpu_pmc_ta.sh <tag> [workload]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-ta}
WL=${2:-dragon1m}
D=gpurun_out/pmc_$TAG
mkdir -p $D
i=0
for set in "TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum TD_TD_BUSY_sum TD_TC_STALL_sum GRBM_GUI_ACTIVE" \
           "TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  RTG_STREAMS=1 timeout -s KILL 300 rocprofv3 --pmc $set --kernel-trace -d $D/p$i -o p$i --output-format csv -- \
      python3 bench.py --steps 1 --warmup 0 --no-cpu --workload $WL > $D/p$i.out 2> $D/p$i.err \
      || { echo "pmc pass $i failed"; tail -5 $D/p$i.err; exit 1; }
  echo "pmc pass $i done"
done
python3 scripts/pmc_counters.py $D $D/ta_$WL.csv $D/ta_$WL.json $WL
rm -rf $D/p[1-9]
