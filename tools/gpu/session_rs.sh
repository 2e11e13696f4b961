#!/bin/bash
# radix sort with block-major tile histograms: GPU tests, then same-box A/B vs the previous library
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> gpurun_out/steps.txt; [ $rc -eq 0 ] || exit $rc
VARIANTS="build_base build" REPS=4 timeout -k 10 400 bash tools/gpu/ab_multi.sh > gpurun_out/ab.log 2>&1; echo "ab rc=$?" >> gpurun_out/steps.txt
