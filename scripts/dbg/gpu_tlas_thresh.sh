set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out/tt
for w in cornell_pt cornell bunny dragon1m; do for t in off on; do
  timeout -k 10 300 python3 bench.py --no-cpu --workload $w --tlas $t --steps 3 > gpurun_out/tt/b_${w}_$t.json 2> gpurun_out/tt/b_${w}_$t.err || { tail -20 gpurun_out/tt/b_${w}_$t.err; exit 1; }
  python3 -c "import json; j=json.load(open('gpurun_out/tt/b_${w}_$t.json')); print('$w $t', j['ms_per_step'], j['config']['tlas_nodes'], j['kernel_ms_rank0_streams1'])"
done; done
