set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out/tu
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_tlas.py -x -q --timeout 300 --timeout-method thread > gpurun_out/tu/test.log 2>&1 || { tail -40 gpurun_out/tu/test.log; exit 1; }
tail -1 gpurun_out/tu/test.log
for c in spheres:auto cornell_pt:on cornell:on dragon1m:on; do
  w=${c%%:*}; t=${c##*:}
  timeout -k 10 300 python3 bench.py --no-cpu --workload $w --tlas $t --steps 3 > gpurun_out/tu/b_${w}_$t.json 2> gpurun_out/tu/b_${w}_$t.err || { tail -20 gpurun_out/tu/b_${w}_$t.err; exit 1; }
  python3 -c "import json; j=json.load(open('gpurun_out/tu/b_${w}_$t.json')); print('$w $t', j['ms_per_step'], j['config']['tlas_nodes'], j['kernel_ms_rank0_streams1'])"
done
