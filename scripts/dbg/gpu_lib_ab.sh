# A/B of library variants on the bench (dragon unless BENCH_ARGS): LIBS="librtg w5 ..."
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out/ab
for lib in ${LIBS:-librtg}; do
  RTG_LIBRARY=raytracer-795_amd/rtg/$lib.so timeout -k 10 300 python3 bench.py --no-cpu --steps 5 $BENCH_ARGS > gpurun_out/ab/b_$lib.json 2> gpurun_out/ab/b_$lib.err || { tail -30 gpurun_out/ab/b_$lib.err; exit 1; }
  python3 -c "import json; j=json.load(open('gpurun_out/ab/b_$lib.json')); print('$lib', j['ms_per_step'], j['kernel_ms_rank0_streams1'])"
done
