#!/bin/bash
# Copy the judged evidence of a gpu_bench_profile.sh run into profiles/ (tracked).
set -e
TAG=$1
D=gpurun_out/prof_$TAG
cp $D/bench.json profiles/${TAG}_bench.json
python3 - "$D/kt/kt_kernel_stats.csv" > profiles/${TAG}_kernel_stats.txt <<'PY'
import csv, sys
print(f"{'kernel':48s} {'calls':>6s} {'total_ms':>10s} {'avg_us':>9s} {'pct':>6s}")
for r in csv.DictReader(open(sys.argv[1])):
    print(f"{r['Name'].split('(')[0].replace('void ', '')[:48]:48s} {r['Calls']:>6s} "
          f"{float(r['TotalDurationNs'])/1e6:10.2f} {float(r['AverageNs'])/1e3:9.1f} {float(r['Percentage']):6.2f}")
# combined closest-hit line (GEN=true level-0 + GEN=false secondary launches), the kernel
# bench.py's roofline.avg_launch_ms averages over
ks = [r for r in csv.DictReader(open(sys.argv[1])) if r['Name'].startswith('void rtg::k_trace<false, false')
      or r['Name'].startswith('rtg::k_trace<false, false')]
if ks:
    c = sum(int(r['Calls']) for r in ks); t = sum(float(r['TotalDurationNs']) for r in ks)
    print(f"{'rtg::k_trace<false, false, *> (combined)':48s} {c:6d} {t/1e6:10.2f} {t/c/1e3:9.1f}")
PY
cp $D/kt/kt_kernel_stats.csv profiles/${TAG}_kernel_stats.csv
python3 scripts/pmc_traffic.py $D profiles/${TAG}_pmc_traffic.json \
    "rocprofv3 --pmc FETCH_SIZE|WRITE_SIZE --kernel-trace -- python3 bench.py --steps 1 --warmup 0 --no-cpu"
cp profiles/${TAG}_pmc_traffic.json profiles/traffic_current.json
