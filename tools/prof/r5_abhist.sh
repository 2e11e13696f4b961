#!/bin/bash
# first radix pass's histogram counted in the pack kernel: parity tests, single-device and sharded A/B
set -u
mkdir -p gpurun_out/shard_ab
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sharded.py tests/test_gpu_slices.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/hist_tests.log 2>&1
rc=$?; tail -3 gpurun_out/hist_tests.log; [ $rc -eq 0 ] || exit $rc
rm -f gpurun_out/ab.txt gpurun_out/shard_ab/ab.txt
VARIANTS="build:SA_HIST_IN_PACK=0 build" REPS=3 bash tools/prof/ab.sh && cat gpurun_out/ab.txt
VARIANTS="build:SA_HIST_IN_PACK=0 build" REPS=2 bash tools/prof/shard_ab.sh
