#!/bin/bash
# One GPU call: the GPU test suite, smoke(), and bench lines for the workloads in $WLS (default: the
# headline dragon1m).  Every step under its own time limit; the chain stops at the first failure.
#   gpurun -- bash scripts/gpu_check.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-check}
D=gpurun_out/$TAG
mkdir -p $D
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread ${PYTEST_ARGS} > $D/gputest.log 2>&1 \
    || { tail -40 $D/gputest.log; exit 1; }
  tail -2 $D/gputest.log
  timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1 || { tail -20 $D/smoke.log; exit 1; }
  cat $D/smoke.log
fi
[ -n "$SKIP_BENCH" ] && { echo done; exit 0; }
for wl in ${WLS:-dragon1m}; do
  timeout -k 10 600 python3 bench.py --workload $wl $BENCH_ARGS > $D/bench_$wl.json 2> $D/bench_$wl.err \
    || { tail -20 $D/bench_$wl.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('$D/bench_$wl.json')); print('$wl', d['ms_per_step'], 'ms', d['value'], 'Mray/s', 'parity', (d.get('parity') or {}).get('differing'), 'k_ms', d['kernel_ms_rank0_streams1'])"
done
echo done
