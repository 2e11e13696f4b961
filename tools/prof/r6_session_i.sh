#!/bin/bash
# Round 6: the sharded reduce's second tier and density-sized pair-count items --
# sharded tests, the real-density test, the configs[3] real-density bench and the
# bench-shape sharded bench (phase clocks).
set -u
mkdir -p gpurun_out/r6i
SA_TEST_RECORD_DIR=gpurun_out/r6i/rec OUT=r6i TESTS="tests/test_gpu_sharded.py tests/test_gpu_big_slices.py" \
    K="sharded or real_density or k12_eight" EXTRA="-s" SECS=700 PER=400 bash tools/prof/r6_tests.sh || exit 1
SA_DEBUG_PHASES=1 timeout -k 10 400 python bench.py --shards 8 --serial-shards --lean --reads 1250000 --steps 3 \
    --warmup 1 --no-cpu-baseline --align-steps 1 --stage-steps 1 > gpurun_out/r6i/c3real.log 2>&1 || exit 1
SA_DEBUG_PHASES=1 timeout -k 10 300 python bench.py --shards 8 --serial-shards --steps 4 --warmup 1 --no-cpu-baseline \
    --align-steps 1 --stage-steps 1 > gpurun_out/r6i/sh8.log 2>&1 || exit 1
for f in c3real sh8; do tail -1 gpurun_out/r6i/$f.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["stage_ms_per_step"], d["shard_info"], d["first_build_ms"])'; done
