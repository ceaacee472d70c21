#!/bin/bash
# Round-end rehearsal of what the driver runs: GPU suite, smoke(), the default bench line, and the
# N>1 bench path rehearsed on one GPU (2 ranks, gloo gather, RTG_BENCH_REHEARSE=1).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
D=gpurun_out/final_check
mkdir -p $D
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $D/tests.log 2>&1 || { tail -30 $D/tests.log; exit 1; }
tail -1 $D/tests.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1 || { tail -20 $D/smoke.log; exit 1; }
tail -2 $D/smoke.log
timeout -k 10 300 python3 bench.py > $D/bench.json 2> $D/bench.err || { tail -20 $D/bench.err; exit 1; }
tail -c 300 $D/bench.json
RTG_BENCH_REHEARSE=1 timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu > $D/rehearse2.json 2> $D/rehearse2.err || { tail -20 $D/rehearse2.err; exit 1; }
python3 -c "import json; d=json.loads(open('$D/rehearse2.json').read().strip().splitlines()[-1]); print('rehearse N=2', d['ms_per_step'], d['value'], d.get('multi'))"
echo final-check-done
