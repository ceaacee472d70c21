#!/bin/bash
# A/B of library variants (rtg/<lib>.so) and level loops on the dragon1m frame: per-rank shard times
# (scripts/shard_probe.py) and, with RTG_KT=1, per-kernel times of a serialised frame.
#   CFGS="lib:loop:waves ..." NS="1 8" bash scripts/gpu_ab2.sh
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
  IFS=: read -r lib mode waves <<< "$cfg"
  echo "== $lib loop=$mode waves=$waves" >> gpurun_out/ab2.log
  RTG_LIBRARY=raytracer-795_amd/rtg/$lib.so RTG_LEVEL_LOOP=$mode RTG_DD_WAVES=$waves RTG_KT=${KT:-1} \
      timeout -k 10 300 python3 scripts/shard_probe.py ${NS:-1 8} >> gpurun_out/ab2.log 2>&1 \
      || { tail -20 gpurun_out/ab2.log; exit 1; }
done
grep -v amdgpu.ids gpurun_out/ab2.log
