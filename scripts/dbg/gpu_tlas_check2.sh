set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out/t
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_tlas.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t/tlas.log 2>&1 || { tail -60 gpurun_out/t/tlas.log; exit 1; }
tail -3 gpurun_out/t/tlas.log
timeout -k 10 900 python3 -u scripts/dbg/tlas_diff.py 64 > gpurun_out/t/tlas_diff.log 2>&1 || { tail -30 gpurun_out/t/tlas_diff.log; exit 1; }
tail -8 gpurun_out/t/tlas_diff.log
timeout -k 10 600 python3 bench.py --no-cpu --workload spheres > gpurun_out/t/bench_spheres.json 2> gpurun_out/t/bench_spheres.err || { tail -30 gpurun_out/t/bench_spheres.err; exit 1; }
cut -c1-700 gpurun_out/t/bench_spheres.json
