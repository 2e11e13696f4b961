#!/bin/bash
# Round 6: the configs[3] real-density test with its record, then the configs[3] real-density
# profile (8 lean virtual shards: kernel stats + PMC passes, traces trimmed after summary).
set -u
mkdir -p gpurun_out/r6h
SA_TEST_RECORD_DIR=gpurun_out/r6h/rec OUT=r6h TESTS="tests/test_gpu_big_slices.py" K="real_density" \
    EXTRA="-s" SECS=500 PER=400 bash tools/prof/r6_tests.sh || exit 1
mv gpurun_out/r6h/tests.log gpurun_out/r6h/tests_real_density.log
SP_TRIM=1 bash tools/prof/slice_prof.sh c3real --reads 1250000 --shards 8 --serial-shards --lean --steps 2 --warmup 1 \
    --align-steps 1 --stage-steps 1 || exit 1
tail -8 gpurun_out/steps.txt
