#!/bin/bash
# One GPU call: the bench's N>1 path rehearsed on one GPU (RTG_BENCH_REHEARSE=1: every rank on cuda:0,
# gloo gather through host memory) for the BASELINE configs' own GPU counts -- C4 cornell on 2 ranks,
# C5 cornell_pt on 8.  Each line carries multi.gathered_equals_single and per-rank shard ms.
#   gpurun -- bash scripts/gpu_rehearse.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/${1:-rehearse}
mkdir -p $D
export RTG_BENCH_REHEARSE=1 MASTER_ADDR=127.0.0.1
run() {   # <workload> <ranks> <port>
  timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node $2 --master-addr 127.0.0.1 \
      --master-port $3 bench.py --workload $1 --gpus $2 --steps 2 --warmup 1 --no-cpu \
      > $D/rehearse_$1_$2.json 2> $D/rehearse_$1_$2.err || { tail -20 $D/rehearse_$1_$2.err; return 1; }
  python3 -c "import json; d=json.load(open('$D/rehearse_$1_$2.json')); m=d['multi']; print('$1', d['n_gpus'], d['ms_per_step'], 'ms', m['gathered_equals_single'], m['shard_ms_per_rank'], m['gather_ms_max_over_ranks'])"
}
run cornell 2 29531 && run cornell_pt 8 29532 && echo done
