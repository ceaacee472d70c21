set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/c11
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_sah.py -x -q --timeout 120 --timeout-method thread > gpurun_out/c11/sah.log 2>&1 || { tail -60 gpurun_out/c11/sah.log; exit 1; }
tail -2 gpurun_out/c11/sah.log
RTG_BUILD_TIMING=1 timeout -k 10 300 python3 scripts/create_probe.py 4 > gpurun_out/c11/create.txt 2>&1 || { tail -30 gpurun_out/c11/create.txt; exit 1; }
grep "^{" gpurun_out/c11/create.txt | cut -c1-330
grep "gpu sah\|sah_\|early\|phase upload\|phase traversal" gpurun_out/c11/create.txt | tail -24
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/c11/gputest.log 2>&1 || { tail -40 gpurun_out/c11/gputest.log; exit 1; }
tail -2 gpurun_out/c11/gputest.log
