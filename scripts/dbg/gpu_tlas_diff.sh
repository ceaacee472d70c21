cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out/d
timeout -k 10 900 python3 -u scripts/dbg/tlas_diff.py ${1:-64} > gpurun_out/d/tlas_diff.log 2>&1; rc=$?; cat gpurun_out/d/tlas_diff.log | tail -40; exit $rc
