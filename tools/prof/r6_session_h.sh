#!/bin/bash
# Round 6: strict-id (Trove replay) GPU tests, the two real-density sharded tests with their
# records, then the configs[3] real-density profile (8 lean virtual shards: kernel stats +
# PMC passes).
set -u
mkdir -p gpurun_out/r6h
OUT=r6h TESTS="tests/test_gpu_parity.py tests/test_gpu_scale.py" K="crp177 or ruddii or strict" \
    SECS=500 PER=300 bash tools/prof/r6_tests.sh || exit 1
mv gpurun_out/r6h/tests.log gpurun_out/r6h/tests_strict.log
SA_TEST_RECORD_DIR=gpurun_out/r6h/rec OUT=r6h TESTS="tests/test_gpu_big_slices.py" K="real_density or k12_eight" \
    EXTRA="-s" SECS=500 PER=400 bash tools/prof/r6_tests.sh || exit 1
mv gpurun_out/r6h/tests.log gpurun_out/r6h/tests_real_density.log
bash tools/prof/slice_prof.sh c3real --reads 1250000 --shards 8 --serial-shards --lean --steps 2 --warmup 1 \
    --align-steps 1 --stage-steps 1 || exit 1
tail -6 gpurun_out/steps.txt
