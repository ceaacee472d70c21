cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out/d
timeout -k 10 900 python3 -u scripts/dbg/tlas_rays.py ${1:-519} > gpurun_out/d/tlas_rays.log 2>&1; rc=$?; tail -60 gpurun_out/d/tlas_rays.log; exit $rc
