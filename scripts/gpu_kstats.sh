#!/bin/bash
# Kernel-time breakdown of bench frames (rocprofv3 kernel trace + stats).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-ks}
mkdir -p gpurun_out/$TAG
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$TAG -o ks --output-format csv -- \
    python3 scripts/frame.py ${2:-3} > gpurun_out/$TAG/out.txt 2> gpurun_out/$TAG/err.txt || { tail -5 gpurun_out/$TAG/err.txt; exit 1; }
cat gpurun_out/$TAG/out.txt
f=$(find gpurun_out/$TAG -name "*kernel_stats.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows:
    print(f"{r['Name'][:60]:60s} calls {r['Calls']:>6s} total_ms {float(r['TotalDurationNs'])/1e6:9.2f} avg_us {float(r['AverageNs'])/1e3:9.1f} pct {float(r['Percentage']):6.2f}")
PY
