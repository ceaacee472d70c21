#!/bin/bash
# A/B of librtg variants on the N-GPU row shards (scripts/shard_probe.py, one shard at a time on
# one GPU): LIBS="a b" NS="1 8" bash scripts/gpu_ab_shard.sh   (after gpu_ab3.sh in the same call)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
: > gpurun_out/ab_shard.log
for rep in 1 2; do
  for lib in ${LIBS:-librtg}; do
    echo "lib=$lib" >> gpurun_out/ab_shard.log
    RTG_LIBRARY=raytracer-795_amd/rtg/$lib.so timeout -k 10 300 python3 scripts/shard_probe.py ${NS:-1 8} \
      >> gpurun_out/ab_shard.log 2>/dev/null || { echo "shard_probe failed: $lib"; exit 1; }
  done
done
cat gpurun_out/ab_shard.log
