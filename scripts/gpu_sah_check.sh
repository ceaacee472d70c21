# SAH traversal tree: parity (SAH + reference tree), then dragon ms/frame with each tree.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out/sah
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_sah.py tests/test_gpu_parity.py -x -q --timeout 180 --timeout-method thread > gpurun_out/sah/test.log 2>&1 || { tail -60 gpurun_out/sah/test.log; exit 1; }
tail -3 gpurun_out/sah/test.log
for m in 1 0; do
  RTG_SAH=$m timeout -k 10 300 python3 bench.py --no-cpu --steps 5 > gpurun_out/sah/bench_sah$m.json 2> gpurun_out/sah/bench_sah$m.err || { tail -30 gpurun_out/sah/bench_sah$m.err; exit 1; }
  python3 -c "import json,sys; j=json.load(open('gpurun_out/sah/bench_sah$m.json')); print('sah=$m', j['ms_per_step'], j['value'])"
done
