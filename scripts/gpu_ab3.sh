#!/bin/bash
# A/B of librtg variants (raytracer-795_amd/rtg/<lib>.so) with scripts/ab.py, each library run
# twice in alternation (A B A B) on $WL (default dragon1m); optional $TESTS first (default library).
#   LIBS="librtg nocert" WL=dragon1m TESTS="tests/test_gpu_parity.py" bash scripts/gpu_ab3.sh
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
  for lib in ${LIBS:-librtg}; do
    for wl in ${WL:-dragon1m}; do
      RTG_LIBRARY=raytracer-795_amd/rtg/$lib.so timeout -k 10 300 python3 scripts/ab.py $wl >> gpurun_out/ab3.log 2>/dev/null \
        || { echo "ab.py failed: $lib $wl"; exit 1; }
    done
  done
done
cat gpurun_out/ab3.log
