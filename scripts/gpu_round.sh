#!/bin/bash
# One GPU call of a profiling round: GPU tests, the official bench line, the rocprofv3
# kernel-trace summary and the PMC counter passes behind the per-kernel rooflines.
#   gpurun -- bash scripts/gpu_round.sh <tag>      then (container) scripts/save_round.sh <tag>
# Every step runs under its own time limit and the chain stops at the first failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-r2}
D=gpurun_out/prof_$TAG
mkdir -p $D
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $D/gputest.log 2>&1 \
    || { tail -40 $D/gputest.log; exit 1; }
  tail -2 $D/gputest.log
fi
timeout -k 10 600 python3 bench.py $BENCH_ARGS > $D/bench.json 2> $D/bench.err || { tail -20 $D/bench.err; exit 1; }
cat $D/bench.json
# kernel trace: passes serialised (--streams 1) so every launch is timed alone
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $D/kt -o kt --output-format csv -- \
    python3 bench.py --no-cpu --streams 1 $BENCH_ARGS > $D/bench_kt.json 2> $D/bench_kt.err || { tail -20 $D/bench_kt.err; exit 1; }
echo "kernel trace done"
# PMC passes (one counter set per run: at most 8 SQ, 4 TCC, 4 TCP, 2 GRBM counters)
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_INSTS_BRANCH GRBM_GUI_ACTIVE" \
           "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU_TRANS_F32 SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_SCA SQ_INST_LEVEL_VMEM" \
           "TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_WRITE_REQ_sum" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 300 rocprofv3 --pmc $set --kernel-trace -d $D/p$i -o p$i --output-format csv -- \
      python3 bench.py --steps 1 --warmup 0 --no-cpu --streams 1 $BENCH_ARGS > $D/p$i.out 2> $D/p$i.err \
      || { echo "pmc pass $i failed"; tail -5 $D/p$i.err; exit 1; }
  echo "pmc pass $i done"
done
echo done
