# fused trace+shade: GPU tests, then dragon ms/frame with RTG_FOLD=1 / 0
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out/fold
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > gpurun_out/fold/test.log 2>&1 || { tail -60 gpurun_out/fold/test.log; exit 1; }
tail -2 gpurun_out/fold/test.log
for f in 1 0; do
  RTG_FOLD=$f timeout -k 10 300 python3 bench.py --no-cpu --steps 5 > gpurun_out/fold/bench_$f.json 2> gpurun_out/fold/bench_$f.err || { tail -30 gpurun_out/fold/bench_$f.err; exit 1; }
  python3 -c "import json; j=json.load(open('gpurun_out/fold/bench_$f.json')); print('fold=$f', j['ms_per_step'], j['value'], j['kernel_ms_rank0_streams1'])"
done
