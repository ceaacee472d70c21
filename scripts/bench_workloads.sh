#!/bin/bash
# One GPU box call: the default bench line (dragon1m) plus the other BASELINE configs' scenes and
# the many-object spheres workload with and without the top-level BVH.
# Usage (on the box): scripts/bench_workloads.sh <tag>   -> gpurun_out/bench_<tag>_<workload>.json
set -e
tag=${1:-dev}
mkdir -p gpurun_out
timeout -k 10 300 python3 -u bench.py --no-cpu > gpurun_out/bench_${tag}_dragon1m.json 2> gpurun_out/bench_${tag}_dragon1m.log
for w in cornell_pt cornell bunny spheres; do
  timeout -k 10 300 python3 -u bench.py --no-cpu --workload $w > gpurun_out/bench_${tag}_$w.json 2> gpurun_out/bench_${tag}_$w.log
done
timeout -k 10 300 python3 -u bench.py --no-cpu --workload spheres --tlas off --steps 2 > gpurun_out/bench_${tag}_spheres_notlas.json 2> gpurun_out/bench_${tag}_spheres_notlas.log
