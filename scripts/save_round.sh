#!/bin/bash
# Copy the judged evidence of a gpu_round.sh run into profiles/ (tracked):
#   <tag>_bench.json            the bench.py line
#   <tag>_kernel_stats.{csv,txt} rocprofv3 --kernel-trace --stats of bench.py --streams 1
#   <tag>_counters.csv          per-kernel PMC counters (dispatches, sum, per-dispatch mean)
#   counters_<workload>.json    the per-dispatch means bench.py's rooflines divide by live launch times
#                               (counters_current.json: the same for the headline workload, dragon1m)
set -e
TAG=$1
WL=${2:-dragon1m}
D=gpurun_out/prof_$TAG
# the bench line re-run with the counters just measured (gpu_profile_all.sh), else the first one
B=$D/bench_final.json; [ -s $B ] || B=$D/bench.json
cp $B profiles/${TAG}_bench.json
python3 - "$D/kt/kt_kernel_stats.csv" > profiles/${TAG}_kernel_stats.txt <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
print(f"{'kernel':48s} {'calls':>6s} {'total_ms':>10s} {'avg_us':>9s} {'pct':>6s}")
for r in rows:
    nm = r['Name'].replace('(anonymous namespace)::', '').replace('void ', '').split('(')[0]
    print(f"{nm[:48]:48s} {r['Calls']:>6s} "
          f"{float(r['TotalDurationNs'])/1e6:10.2f} {float(r['AverageNs'])/1e3:9.1f} {float(r['Percentage']):6.2f}")
# combined closest-hit line (GEN=true level-0 + GEN=false secondary launches): the kernel whose
# average bench.py's roofline.avg_launch_ms measures
for pre in ('rtg::k_trace<false, false', 'rtg::k_shade<false, false, 512, false'):
    ks = [r for r in rows if r['Name'].replace('void ', '').startswith(pre + ',')]
    if ks:
        c = sum(int(r['Calls']) for r in ks); t = sum(float(r['TotalDurationNs']) for r in ks)
        print(f"{pre + ', *> (combined)':48s} {c:6d} {t/1e6:10.2f} {t/c/1e3:9.1f}")
PY
cp $D/kt/kt_kernel_stats.csv profiles/${TAG}_kernel_stats.csv
if [ -f $D/counters_$WL.json ]; then     # extracted on the GPU box (gpu_profile_all.sh drops the raw CSVs)
  cp $D/counters_$WL.csv profiles/${TAG}_counters.csv; cp $D/counters_$WL.json profiles/${TAG}_counters.json
else
  python3 scripts/pmc_counters.py $D profiles/${TAG}_counters.csv profiles/${TAG}_counters.json $WL
fi
cp profiles/${TAG}_counters.json profiles/counters_${WL}.json
[ "$WL" = dragon1m ] && cp profiles/${TAG}_counters.json profiles/counters_current.json
echo saved $TAG
