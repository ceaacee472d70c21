set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out/sah
for m in 1 0; do
  RTG_STREAMS=1 RTG_SAH=$m RTG_LIBRARY=raytracer-795_amd/rtg/${LIB:-dbg_nopk}.so timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_BRANCH --kernel-trace -d gpurun_out/sah/pmc_$m -o p --output-format csv -- python3 scripts/probe.py dragon1m 16 > gpurun_out/sah/pmc_$m.log 2>&1 || { tail -30 gpurun_out/sah/pmc_$m.log; exit 1; }
  f=$(find gpurun_out/sah/pmc_$m -name "*counter_collection.csv" | head -1)
  echo "== RTG_SAH=$m"; python3 - "$f" <<'P'
import csv, sys, collections
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Kernel_Name"]
    if "k_trace" not in n and "k_shadow" not in n: continue
    if "true, true" in n or "true," in n.split("<")[1][:12] and "false, true" in n[:40]: pass
    agg[n[:55]][r["Counter_Name"]] += float(r["Counter_Value"])
for n, c in agg.items():
    print(n, {k: f"{v:.3g}" for k, v in sorted(c.items())})
P
done
