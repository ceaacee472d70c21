#!/bin/bash
# Round-3 check: GPU test suite, the bench line (parity + rooflines), and the 1-rank RCCL bench
# path (rtg_render_ranked, gathered_equals_single).  Each step has its own time limit; the chain
# stops at the first failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-r3a}
D=gpurun_out/$TAG
mkdir -p $D
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread $PYTEST_ARGS > $D/gputest.log 2>&1 \
    || { tail -60 $D/gputest.log; exit 1; }
  grep -E "passed|failed" $D/gputest.log | tail -2
  grep -E "Linf|differing|rays \{" $D/gputest.log | head -20
fi
timeout -k 10 600 python3 bench.py $BENCH_ARGS > $D/bench.json 2> $D/bench.err || { tail -20 $D/bench.err; exit 1; }
cat $D/bench.json
if [ -z "$SKIP_RANKED" ]; then
  timeout -k 10 300 python3 bench.py --ranked --no-cpu --steps 2 $BENCH_ARGS > $D/bench_ranked.json 2> $D/bench_ranked.err \
    || { tail -20 $D/bench_ranked.err; exit 1; }
  python3 -c "import json;d=json.load(open('$D/bench_ranked.json'));print('ranked', d['ms_per_step'], d['multi'])"
fi
echo done
