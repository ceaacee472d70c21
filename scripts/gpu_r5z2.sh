set -o pipefail
cd "$GRAFT_REPO_ROOT"
WLS="spheres" bash scripts/gpu_profile_all.sh r5z && mkdir -p gpurun_out/r5z_fix && timeout -k 10 600 python3 bench.py --workload cornell > gpurun_out/r5z_fix/cornell_bench_final.json 2> gpurun_out/r5z_fix/cornell.err && tail -c 300 gpurun_out/r5z_fix/cornell_bench_final.json
