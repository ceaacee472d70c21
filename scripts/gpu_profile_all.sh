#!/bin/bash
# One GPU call: gpu_round.sh (bench line, kernel trace, PMC passes; tests skipped) for every
# workload in $WLS, tags <prefix>_<workload>.  Then, in the container:
#   for w in $WLS; do scripts/save_round.sh <prefix>_$w $w; done
set -o pipefail
cd "$GRAFT_REPO_ROOT"
P=${1:-r3c}
for wl in ${WLS:-dragon1m cornell cornell_pt bunny}; do
  echo "=== $wl"
  SKIP_TESTS=1 BENCH_ARGS="--workload $wl $EXTRA_ARGS" bash scripts/gpu_round.sh ${P}_$wl > gpurun_out/prof_${P}_$wl.txt 2>&1 \
    || { tail -20 gpurun_out/prof_${P}_$wl.txt; exit 1; }
  tail -1 gpurun_out/prof_${P}_$wl.txt
  # the counters just measured, then the bench line again with them (frame HBM, per-kernel rooflines)
  python3 scripts/pmc_counters.py gpurun_out/prof_${P}_$wl gpurun_out/prof_${P}_$wl/counters_$wl.csv \
      gpurun_out/prof_${P}_$wl/counters_$wl.json $wl || exit 1
  # the raw per-dispatch CSVs are tens of MB per workload (gpurun copies back <= 64 MiB): keep the
  # per-kernel summaries only
  rm -rf gpurun_out/prof_${P}_$wl/p[1-9] gpurun_out/prof_${P}_$wl/kt/kt_kernel_trace.csv
  RTG_COUNTERS_DIR=gpurun_out/prof_${P}_$wl timeout -k 10 600 python3 bench.py --workload $wl $EXTRA_ARGS \
      > gpurun_out/prof_${P}_$wl/bench_final.json 2> gpurun_out/prof_${P}_$wl/bench_final.err || exit 1
  tail -c 400 gpurun_out/prof_${P}_$wl/bench_final.json
done
