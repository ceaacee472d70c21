set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out/tl
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_tlas.py tests/test_gpu_parity.py -x -q --timeout 180 --timeout-method thread > gpurun_out/tl/test.log 2>&1 || { tail -40 gpurun_out/tl/test.log; exit 1; }
tail -1 gpurun_out/tl/test.log
for w in spheres dragon1m; do
  timeout -k 10 300 python3 bench.py --no-cpu --workload $w --steps 5 > gpurun_out/tl/b_$w.json 2> gpurun_out/tl/b_$w.err || { tail -20 gpurun_out/tl/b_$w.err; exit 1; }
  python3 -c "import json; j=json.load(open('gpurun_out/tl/b_$w.json')); print('$w', j['ms_per_step'], j['kernel_ms_rank0_streams1'])"
done
