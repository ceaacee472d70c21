#!/bin/bash
# GPU check used during development: parity tests, then a short bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests/test_gpu_parity.py -q -m gpu --maxfail=5 -k "not pruned_equals" > gpurun_out/pytest1.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest1.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest crashed rc=$rc"; exit $rc; fi
timeout -k 10 600 python bench.py --steps 2 --warmup 1 --cpu-rows 1 > gpurun_out/bench1.json 2> gpurun_out/bench1.err
echo "bench rc=$?"
