#!/bin/bash
# One GPU box call: the default bench line (dragon1m) plus the other BASELINE configs' scenes.
# Usage (on the box): scripts/bench_workloads.sh <tag>   -> gpurun_out/bench_<tag>_<workload>.json
set -e
tag=${1:-dev}
mkdir -p gpurun_out
timeout -k 10 300 python3 -u bench.py --no-cpu > gpurun_out/bench_${tag}_dragon1m.json 2> gpurun_out/bench_${tag}_dragon1m.log
for w in cornell_pt cornell bunny; do
  timeout -k 10 300 python3 -u bench.py --no-cpu --workload $w > gpurun_out/bench_${tag}_$w.json 2> gpurun_out/bench_${tag}_$w.log
done
