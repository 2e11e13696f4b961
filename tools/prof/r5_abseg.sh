#!/bin/bash
# phase-1 row segments: parity tests, then same-box A/B of SA_P1_SEGS (0 = one-segment kernel)
set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest ${TESTS:-tests/test_gpu_hoxd.py tests/test_gpu_parity.py} -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/al_tests.log 2>&1
rc=$?; tail -3 gpurun_out/al_tests.log; [ $rc -eq 0 ] || exit $rc
rm -f gpurun_out/ab.txt
VARIANTS="${VARIANTS:-build:SA_P1_SEGS=0 build build:SA_P1_SEGS=2 build:SA_P1_SEGS=8}" REPS=3 bash tools/prof/ab.sh; cat gpurun_out/ab.txt
