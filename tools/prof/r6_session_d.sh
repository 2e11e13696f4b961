#!/bin/bash
# Round 6: sharded A/B (r5 library vs this tree), default bench, real-density test.
set -u
mkdir -p gpurun_out/r6d
VARIANTS="build_r5 build" REPS=2 ARGS="--shards 8 --serial-shards" AB_TIMEOUT=150 bash tools/prof/ab.sh || exit 1
mv gpurun_out/ab.txt gpurun_out/r6d/ab_sharded8.txt
cat gpurun_out/r6d/ab_sharded8.txt
timeout -k 10 600 python bench.py > gpurun_out/r6d/bench.log 2>&1 || exit 1
tail -1 gpurun_out/r6d/bench.log > gpurun_out/r6d/bench.json
OUT=r6d TESTS="tests/test_gpu_big_slices.py" K="real_density" SECS=600 PER=550 SA_TEST_RECORD_DIR=gpurun_out/r6d/rec bash tools/prof/r6_tests.sh
