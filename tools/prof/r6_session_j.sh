#!/bin/bash
# Round 6: source-relative packed values -- the sharded tests with the mode forced
# (SA_SRC_REL=1), the real-density test (where it is the default), the configs[3]
# real-density bench and the bench-shape sharded bench.
set -u
mkdir -p gpurun_out/r6j
SA_SRC_REL=1 OUT=r6j TESTS="tests/test_gpu_sharded.py" SECS=400 PER=300 bash tools/prof/r6_tests.sh || exit 1
mv gpurun_out/r6j/tests.log gpurun_out/r6j/tests_srcrel.log
SA_TEST_RECORD_DIR=gpurun_out/r6j/rec OUT=r6j TESTS="tests/test_gpu_big_slices.py" K="real_density or k12_eight" \
    EXTRA="-s" SECS=500 PER=400 bash tools/prof/r6_tests.sh || exit 1
SA_DEBUG_PHASES=1 timeout -k 10 400 python bench.py --shards 8 --serial-shards --lean --reads 1250000 --steps 3 \
    --warmup 1 --no-cpu-baseline --align-steps 1 --stage-steps 1 > gpurun_out/r6j/c3real.log 2>&1 || exit 1
SA_DEBUG_PHASES=1 timeout -k 10 300 python bench.py --shards 8 --serial-shards --steps 4 --warmup 1 --no-cpu-baseline \
    --align-steps 1 --stage-steps 1 > gpurun_out/r6j/sh8.log 2>&1 || exit 1
for f in c3real sh8; do tail -1 gpurun_out/r6j/$f.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["stage_ms_per_step"], d["shard_info"], d["first_build_ms"])'; done
