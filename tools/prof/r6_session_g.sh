#!/bin/bash
# Round 6: sharded tests + the two real-density tests, then the 2 x 1.25M rank-size
# profile (kernel stats + FETCH/WRITE/SQ/LDS PMC).
set -u
mkdir -p gpurun_out/r6g
OUT=r6g TESTS="tests/test_gpu_sharded.py tests/test_gpu_big_slices.py" K="sharded or real_density or k12_eight" \
    SECS=700 PER=400 bash tools/prof/r6_tests.sh || exit 1
bash tools/prof/slice_prof.sh rank2 --reads 1250000 --shards 2 --serial-shards --steps 3 --warmup 1 \
    --align-steps 1 --stage-steps 1 || exit 1
tail -3 gpurun_out/steps.txt
