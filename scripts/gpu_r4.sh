#!/bin/bash
# Round-4 GPU call: steps named on the command line, each under its own time limit; the chain
# stops at the first step that faults, aborts or times out (a test failure, rc 1, is reported
# and the call goes on only for later non-test steps when KEEP_GOING=1).
#   gpurun -- bash scripts/gpu_r4.sh <tag> tests bench kt_cornell_pt tl_dragon_shard8 ...
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=$1; shift
D=gpurun_out/$TAG
mkdir -p $D
stop() { echo "step $1 ended with rc $2: stopping"; exit $2; }
run() {   # run <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  local i=2; local base=$name
  while [ -e $D/$name.out ]; do name=${base}_$i; i=$((i+1)); done   # repeated steps keep their outputs
  timeout -k 10 $secs "$@" > $D/$name.out 2> $D/$name.err
  local rc=$?
  echo "[$name] rc=$rc"
  tail -3 $D/$name.out
  if [ $rc -ne 0 ]; then tail -15 $D/$name.err; fi
  if [ $rc -ne 0 ] && { [ $rc -ne 1 ] || [ -z "$KEEP_GOING" ]; }; then stop $name $rc; fi
  return 0
}
for step in "$@"; do
  case $step in
    tests) run tests 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread --durations=20 ;;
    tests_*) run $step 600 python3 -u -m pytest tests/test_gpu_${step#tests_}.py -m gpu -x -q --timeout 300 --timeout-method thread ;;
    bench) run bench 300 python3 bench.py ;;
    bench_*) run $step 400 python3 bench.py --workload ${step#bench_} ;;
    nocpu_*) run $step 300 python3 bench.py --no-cpu --workload ${step#nocpu_} ;;
    hipinit) run hipinit 120 python3 scripts/hip_init_probe.py ;;
    create) run create 300 env RTG_BUILD_TIMING=1 python3 scripts/create_probe.py 3 ;;
    createenv:*) IFS=: read -r _ kv <<< "$step"; n=${kv//=/_}; run create_${n//,/_} 300 env RTG_BUILD_TIMING=1 ${kv//,/ } python3 scripts/create_probe.py 3 ;;
    create_*) run $step 300 env RTG_BUILD_TIMING=1 python3 scripts/create_probe.py 3 ${step#create_} ;;
    shard) run shard 300 python3 scripts/shard_probe.py 1 8 ;;
    eb:*) IFS=: read -r _ kv wl <<< "$step"; name="eb_${kv//=/_}_$wl"
          run $name 300 env $kv python3 bench.py --no-cpu --workload $wl ;;
    lib:*) IFS=: read -r _ lib wl <<< "$step"; run lib_${lib}_$wl 300 env RTG_LIBRARY=raytracer-795_amd/rtg/$lib.so python3 bench.py --no-cpu --workload $wl ;;
    shardenv:*) IFS=: read -r _ kv <<< "$step"; n=${kv//=/_}; run shard_${n//,/_} 300 env ${kv//,/ } python3 scripts/shard_probe.py 1 8 ;;
    kt_*) wl=${step#kt_}; run $step 300 rocprofv3 --kernel-trace --stats -d $D/$step -o kt --output-format csv -- python3 scripts/tl_probe.py $wl 2
          python3 scripts/tl_util.py $(ls $D/$step/*kernel_trace.csv | head -1) > $D/${step}_util.txt; cat $D/${step}_util.txt ;;
    ktshardenv:*) IFS=: read -r _ kv wl <<< "$step"; name="ktshard_${kv//=/_}_$wl"
          run $name 300 env $kv rocprofv3 --kernel-trace --stats -d $D/$name -o kt --output-format csv -- python3 scripts/tl_probe.py $wl 3 0 8
          python3 scripts/tl_util.py $(ls $D/$name/*kernel_trace.csv | head -1) > $D/${name}_util.txt; cat $D/${name}_util.txt ;;
    ktshard_*) wl=${step#ktshard_}; run $step 300 rocprofv3 --kernel-trace --stats -d $D/$step -o kt --output-format csv -- python3 scripts/tl_probe.py $wl 3 0 8
          python3 scripts/tl_util.py $(ls $D/$step/*kernel_trace.csv | head -1) > $D/${step}_util.txt; cat $D/${step}_util.txt ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo "all steps done"
