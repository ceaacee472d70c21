#!/bin/bash
# A/B of librtg variants on one GPU box (dev tool): scripts/ab.py for every (round, workload, variant),
# variants interleaved so box drift hits them alike.  Variants are raytracer-795_amd/rtg/<name>.so
# (scripts/build_variant.sh, or any build of the tree), selected through RTG_LIBRARY; "<lib>@k=v,k=v" adds
# render options (ab.py AB_OPTS), e.g. librtg@tile_band=8; "<lib>@build:k=v" build options (AB_BUILD), e.g.
# librtg@build:bvh_builder=1.
#   gpurun -- 'VARIANTS="v_base v_cur" WLS="dragon1m cornell_pt" ROUNDS=2 bash scripts/gpu_ab.sh <tag>'
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-ab}
D=gpurun_out/$TAG
mkdir -p $D
for r in $(seq 1 ${ROUNDS:-2}); do
  for wl in ${WLS:-dragon1m}; do
    for v in ${VARIANTS}; do
      lib=${v%%@*}; opt=""; [ "$lib" != "$v" ] && opt=${v#*@}
      bopt=""; case "$opt" in build:*) bopt=${opt#build:}; opt="";; esac
      RTG_LIBRARY=raytracer-795_amd/rtg/$lib.so AB_TAG=$v AB_OPTS=$opt AB_BUILD=$bopt AB_FRAMES=${AB_FRAMES:-5} timeout -k 10 300 \
          python3 scripts/ab.py $wl >> $D/ab.jsonl 2>> $D/ab.err || { tail -5 $D/ab.err; exit 1; }
      tail -1 $D/ab.jsonl | cut -c1-260
    done
  done
done
echo done
