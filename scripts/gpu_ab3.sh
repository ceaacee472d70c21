#!/bin/bash
# A/B of librtg variants (raytracer-795_amd/rtg/<lib>.so) with scripts/ab.py, each library run
# twice in alternation (A B A B) on $WL (default dragon1m); optional $TESTS first (default library).
#   LIBS="librtg nocert librtg:RTG_REFILL=1,RTG_REFILL_MIN=8" WL=dragon1m TESTS="..." bash scripts/gpu_ab3.sh
# (an entry lib:VAR=val,... runs that library with those environment settings)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python3 -u -m pytest $TESTS -m gpu -x -q --timeout 300 --timeout-method thread \
      > gpurun_out/ab3_test.log 2>&1 || { tail -40 gpurun_out/ab3_test.log; exit 1; }
  tail -2 gpurun_out/ab3_test.log
fi
: > gpurun_out/ab3.log
for rep in 1 2; do
  for cfg in ${LIBS:-librtg}; do
    lib=${cfg%%:*}; envs=${cfg#*:}; [ "$envs" = "$cfg" ] && envs=""
    for wl in ${WL:-dragon1m}; do
      env ${envs//,/ } AB_TAG="$cfg" RTG_LIBRARY=raytracer-795_amd/rtg/$lib.so timeout -k 10 300 python3 scripts/ab.py $wl \
        >> gpurun_out/ab3.log 2>/dev/null || { echo "ab.py failed: $cfg $wl"; exit 1; }
    done
  done
done
cat gpurun_out/ab3.log
