set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out/sah
for spp in 16 64; do for m in 1 0; do
  RTG_STREAMS=1 RTG_SAH=$m RTG_LIBRARY=raytracer-795_amd/rtg/${LIB:-dbg_nopk}.so timeout -k 10 300 python3 scripts/probe.py dragon1m $spp > gpurun_out/sah/probe2_$m.log 2>&1 || { tail -30 gpurun_out/sah/probe2_$m.log; exit 1; }
  echo "== spp=$spp RTG_SAH=$m"; grep collect_timing gpurun_out/sah/probe2_$m.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print({k: round(d[k],2) for k in (\"render_ms\",\"trace_ms\",\"shadow_ms\",\"shade_ms\",\"passes\")})"
done; done
