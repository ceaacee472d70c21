#!/bin/bash
# Official bench line + rocprofv3 kernel-trace summary + separate PMC passes (FETCH_SIZE, WRITE_SIZE).
# Afterwards (in the container): scripts/save_profile.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-r1}
mkdir -p gpurun_out/prof_$TAG
timeout -k 10 600 python3 bench.py > gpurun_out/prof_$TAG/bench.json 2> gpurun_out/prof_$TAG/bench.err || exit $?
cat gpurun_out/prof_$TAG/bench.json
RTG_STREAMS=1 timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG/kt -o kt --output-format csv -- \
    python3 bench.py --no-cpu > gpurun_out/prof_$TAG/bench_kt.json 2> gpurun_out/prof_$TAG/bench_kt.err || exit $?
RTG_STREAMS=1 timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/prof_$TAG/fetch -o fetch --output-format csv -- \
    python3 bench.py --steps 1 --warmup 0 --no-cpu > /dev/null 2> gpurun_out/prof_$TAG/fetch.err || exit $?
RTG_STREAMS=1 timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/prof_$TAG/write -o write --output-format csv -- \
    python3 bench.py --steps 1 --warmup 0 --no-cpu > /dev/null 2> gpurun_out/prof_$TAG/write.err || exit $?
echo done
