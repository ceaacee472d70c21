#!/bin/bash
# One GPU call: per-rank shard times (scripts/shard_probe.py) under the default band rule and its
# neighbours, dragon1m and cornell_pt.  Every step under its own limit; the chain stops at a failure.
#   gpurun -- bash scripts/gpu_shards.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/${1:-shards}
mkdir -p $D
P="timeout -k 10 300 python3 scripts/shard_probe.py"
$P 1 2 4 8 >> $D/probe.txt 2>> $D/probe.err || { tail -5 $D/probe.err; exit 1; }
RTG_PROBE_OPTS="tile_band=8" $P 2 4 8 >> $D/probe.txt 2>> $D/probe.err || { tail -5 $D/probe.err; exit 1; }
RTG_PROBE_OPTS="tile_band=32" $P 2 4 8 >> $D/probe.txt 2>> $D/probe.err || { tail -5 $D/probe.err; exit 1; }
RTG_WORKLOAD=cornell_pt $P 1 8 >> $D/probe.txt 2>> $D/probe.err || { tail -5 $D/probe.err; exit 1; }
RTG_WORKLOAD=cornell_pt RTG_PROBE_OPTS="tile_band=16" $P 1 8 >> $D/probe.txt 2>> $D/probe.err || { tail -5 $D/probe.err; exit 1; }
RTG_WORKLOAD=cornell_pt RTG_PROBE_OPTS="tile_band=32" $P 8 >> $D/probe.txt 2>> $D/probe.err || { tail -5 $D/probe.err; exit 1; }
cat $D/probe.txt
