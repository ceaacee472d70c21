set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out/sah
for m in 1 0; do
  RTG_STREAMS=1 RTG_SAH=$m RTG_LIBRARY=raytracer-795_amd/rtg/${LIB:-dbg_nopk}.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/sah/prof_$m -o run --output-format csv -- python3 scripts/probe.py dragon1m 64 > gpurun_out/sah/prof_$m.log 2>&1 || { tail -30 gpurun_out/sah/prof_$m.log; exit 1; }
  f=$(find gpurun_out/sah/prof_$m -name "*kernel_stats.csv" | head -1)
  echo "== RTG_SAH=$m"; python3 - "$f" <<'P'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:8]:
    print(f'{r["Name"][:70]:70s} n={r["Calls"]:>5s} tot={float(r["TotalDurationNs"])/1e6:8.2f}ms avg={float(r["AverageNs"])/1e3:8.1f}us')
P
done
