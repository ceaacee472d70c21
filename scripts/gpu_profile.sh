#!/bin/bash
# rocprofv3 kernel-trace summary of the bench command, then separate PMC passes for HBM bytes.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/kt -o kt --output-format csv -- \
    python3 bench.py --steps 2 --warmup 1 --no-cpu > gpurun_out/prof/bench_kt.json 2> gpurun_out/prof/bench_kt.err || exit $?
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/prof/fetch -o fetch --output-format csv -- \
    python3 bench.py --steps 1 --warmup 0 --no-cpu > gpurun_out/prof/bench_fetch.json 2> gpurun_out/prof/bench_fetch.err || exit $?
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/prof/write -o write --output-format csv -- \
    python3 bench.py --steps 1 --warmup 0 --no-cpu > gpurun_out/prof/bench_write.json 2> gpurun_out/prof/bench_write.err || exit $?
timeout -k 10 900 python -m pytest tests/test_gpu_parity.py -q -m gpu -k "pruned_equals" -s > gpurun_out/pytest_prune.log 2>&1
echo "prune rc=$?"
find gpurun_out/prof -name "*.csv" | head -50
