set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out/sah
for v in librtg dbg_nopk; do
  echo "== $v"
  RTG_LIBRARY=raytracer-795_amd/rtg/$v.so timeout -k 10 300 python3 -u scripts/dbg/sah_diff.py bunny > gpurun_out/sah/$v.log 2>&1 || { tail -30 gpurun_out/sah/$v.log; exit 1; }
  grep -E "mismatches" gpurun_out/sah/$v.log
done
