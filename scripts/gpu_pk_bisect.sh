#!/bin/bash
# Packed-f32 bisection (DESIGN.md §4 "Compiler note", profiles/r3_pk_bisect.txt): tests/test_gpu_sah.py
# against librtg variants built at commit 6ae2d69 (whose rtg_device.hip has the diagnostic macros) with
# packed-f32 ops enabled, e.g. in csrc: make OUT=../rtg/pk1.so OBJ=../../build/pk1 NOPK= EXTRA=-DRTG_PK_ONLY=1
# (packed in one kernel family only) or EXTRA="-DRTG_PK_ONLY=1 -DRTG_PK_FENCE=3" (and not in region 3).  A test failure (exit 1) moves on to the next variant;
# anything else (fault, abort, time limit) ends the script.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for v in ${VARIANTS:-pk0 pk1 pk2 pk3 pk4}; do
  RTG_LIBRARY=raytracer-795_amd/rtg/$v.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_sah.py -m gpu -x -q \
      --timeout 120 --timeout-method thread > gpurun_out/bisect_$v.txt 2>&1
  rc=$?
  echo "$v rc=$rc $(grep -E 'passed|failed' gpurun_out/bisect_$v.txt | tail -1)"
  grep -E "^(FAILED|E  )" gpurun_out/bisect_$v.txt | head -6
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
done
