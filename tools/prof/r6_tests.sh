#!/bin/bash
# Round 6: a GPU test subset (TESTS, -k filter K) into gpurun_out/$OUT/tests.log.
set -u
OUT=${OUT:-r6}
mkdir -p gpurun_out/$OUT
timeout -k 10 ${SECS:-900} python -u -m pytest ${TESTS:-tests/test_gpu_sharded.py} -m gpu -x -v \
    --timeout ${PER:-400} --timeout-method thread ${EXTRA:-} ${K:+-k "$K"} > gpurun_out/$OUT/tests.log 2>&1
rc=$?
tail -5 gpurun_out/$OUT/tests.log
exit $rc
