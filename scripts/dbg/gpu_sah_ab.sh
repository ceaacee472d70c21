# dragon ms/frame: {packed fp32 on, off} x {SAH tree, reference tree}
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out/sah
for lib in ${LIBS:-librtg dbg_nopk}; do
  for m in 1 0; do
    RTG_SAH=$m RTG_LIBRARY=raytracer-795_amd/rtg/$lib.so timeout -k 10 300 python3 bench.py --no-cpu --steps 5 ${BENCH_ARGS:-} > gpurun_out/sah/ab_${lib}_$m.json 2> gpurun_out/sah/ab_${lib}_$m.err || { tail -30 gpurun_out/sah/ab_${lib}_$m.err; exit 1; }
    python3 -c "import json; j=json.load(open('gpurun_out/sah/ab_${lib}_$m.json')); print('$lib sah=$m', j['ms_per_step'], j['value'])"
  done
done
