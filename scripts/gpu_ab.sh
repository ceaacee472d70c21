#!/bin/bash
# A/B timing: pytest -m gpu on the default library, then probe.py for each "lib:streams" config in $CONFIGS.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -q -m gpu --maxfail=3 > gpurun_out/pytest_ab.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_ab.log; [ $rc -ne 0 ] && exit $rc
for c in ${CONFIGS:-librtg:2}; do
  lib=${c%%:*}; ns=${c##*:}
  echo "== $lib streams=$ns"
  RTG_STREAMS=$ns RTG_LIBRARY=raytracer-795_amd/rtg/$lib.so timeout -k 10 200 python scripts/probe.py ${SCENE:-dragon1m} 64 $DEPTH > gpurun_out/ab_$lib_$ns.log 2>&1 || { tail -5 gpurun_out/ab_$lib_$ns.log; exit 1; }
  grep opts gpurun_out/ab_$lib_$ns.log | python3 -c '
import sys, json
for l in sys.stdin:
    d = json.loads(l)
    print("  ", d["opts"], "render %.2f trace %.2f shadow %.2f" % (d["render_ms"], d["trace_ms"], d["shadow_ms"]))'
done
