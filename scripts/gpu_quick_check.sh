set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out/q
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > gpurun_out/q/gputest.log 2>&1 || { tail -60 gpurun_out/q/gputest.log; exit 1; }
tail -3 gpurun_out/q/gputest.log
timeout -k 10 600 python3 bench.py > gpurun_out/q/bench.json 2> gpurun_out/q/bench.err || { tail -30 gpurun_out/q/bench.err; exit 1; }
cat gpurun_out/q/bench.json
