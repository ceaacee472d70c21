#!/bin/bash
# A/B of library variants (rtg/<lib>.so) and environment settings on the dragon1m frame: per-rank
# shard times (scripts/shard_probe.py) and, with KT=1 (default), per-kernel times of a serialised
# frame.   CFGS="lib:VAR=val,VAR=val ..." NS="1 8" bash scripts/gpu_ab2.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python3 -u -m pytest $TESTS -x -q --timeout 120 --timeout-method thread \
      > gpurun_out/ab2_test.log 2>&1 || { tail -40 gpurun_out/ab2_test.log; exit 1; }
  tail -2 gpurun_out/ab2_test.log
fi
: > gpurun_out/ab2.log
for cfg in $CFGS; do
  lib=${cfg%%:*}; envs=${cfg#*:}; [ "$envs" = "$cfg" ] && envs=""
  echo "== $lib $envs" >> gpurun_out/ab2.log
  env ${envs//,/ } RTG_LIBRARY=raytracer-795_amd/rtg/$lib.so RTG_KT=${KT:-1} \
      timeout -k 10 300 python3 scripts/shard_probe.py ${NS:-1 8} >> gpurun_out/ab2.log 2>&1 \
      || { tail -20 gpurun_out/ab2.log; exit 1; }
done
grep -v amdgpu.ids gpurun_out/ab2.log
