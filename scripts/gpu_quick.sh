#!/bin/bash
# GPU parity tests, then the probe (stats + timing) for the default library and any
# variant libraries named in $VARIANTS (dev builds under raytracer-795_amd/rtg/).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests/test_gpu_parity.py -q -m gpu --maxfail=3 > gpurun_out/pytest_q.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_q.log; tail -3 gpurun_out/pytest_q.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python scripts/probe.py ${1:-dragon1m} ${2:-64} > gpurun_out/probe.log 2>&1 || { cat gpurun_out/probe.log; exit 1; }
cat gpurun_out/probe.log
for v in $VARIANTS; do
  echo "== variant $v"
  RTG_LIBRARY=raytracer-795_amd/rtg/$v timeout -k 10 300 python scripts/probe.py ${1:-dragon1m} ${2:-64} > gpurun_out/probe_$v.log 2>&1 || { cat gpurun_out/probe_$v.log; exit 1; }
  cat gpurun_out/probe_$v.log
done
