set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out/t
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t/gputest.log 2>&1 || { tail -80 gpurun_out/t/gputest.log; exit 1; }
tail -3 gpurun_out/t/gputest.log
timeout -k 10 600 python3 bench.py --no-cpu > gpurun_out/t/bench_dragon.json 2> gpurun_out/t/bench_dragon.err || { tail -30 gpurun_out/t/bench_dragon.err; exit 1; }
cat gpurun_out/t/bench_dragon.json | cut -c1-600
timeout -k 10 600 python3 bench.py --no-cpu --workload spheres > gpurun_out/t/bench_spheres.json 2> gpurun_out/t/bench_spheres.err || { tail -30 gpurun_out/t/bench_spheres.err; exit 1; }
cut -c1-600 gpurun_out/t/bench_spheres.json
RTG_TLAS=0 timeout -k 10 900 python3 bench.py --no-cpu --workload spheres --steps 1 --warmup 0 > gpurun_out/t/bench_spheres_notlas.json 2> gpurun_out/t/bench_spheres_notlas.err || { tail -30 gpurun_out/t/bench_spheres_notlas.err; exit 1; }
cut -c1-600 gpurun_out/t/bench_spheres_notlas.json
