#!/bin/bash
# bucket build split: GPU tests on the guarded build first; the A/B only when every test passed
set -u
mkdir -p gpurun_out
timeout -k 10 240 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc" >> gpurun_out/steps.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?; echo "gpu_tests rc=$rc" >> gpurun_out/steps.txt
[ $rc -eq 0 ] || exit $rc
VARIANTS="build_old build_ps6 build_ps7" REPS=3 timeout -k 10 400 bash tools/gpu/ab_multi.sh > gpurun_out/ab.log 2>&1; echo "ab rc=$?" >> gpurun_out/steps.txt
