set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out/st
for n in ${NS:-8 4 2}; do
  RTG_STREAMS=$n timeout -k 10 300 python3 bench.py --no-cpu --steps 5 $BENCH_ARGS > gpurun_out/st/b_$n.json 2> gpurun_out/st/b_$n.err || { tail -20 gpurun_out/st/b_$n.err; exit 1; }
  python3 -c "import json; j=json.load(open('gpurun_out/st/b_$n.json')); print('streams=$n', j['ms_per_step'])"
done
