#!/bin/bash
# Occupancy / issue counters of one bench frame per library variant: one SQ pass + one GRBM pass each.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-occ}
for v in ${VARIANTS:-librtg}; do
  D=gpurun_out/pmc_${TAG}_$v
  mkdir -p $D
  RTG_LIBRARY=raytracer-795_amd/rtg/$v.so timeout -k 10 180 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM \
     --kernel-trace -d $D/p1 -o p1 --output-format csv -- python3 scripts/frame.py 1 > $D/p1.out 2> $D/p1.err || { tail -3 $D/p1.err; exit 1; }
  RTG_LIBRARY=raytracer-795_amd/rtg/$v.so timeout -k 10 180 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT \
     --kernel-trace -d $D/p2 -o p2 --output-format csv -- python3 scripts/frame.py 1 > $D/p2.out 2> $D/p2.err || { tail -3 $D/p2.err; exit 1; }
  echo "== $v"; python3 scripts/pmc_summary.py $D
done
