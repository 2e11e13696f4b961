#!/bin/bash
# sharded parity tests, then same-box per-shard A/B (tools/prof/shard_ab.sh)
set -u
mkdir -p gpurun_out/shard_ab
timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_gpu_sharded.py} -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/shard_ab/tests.log 2>&1
rc=$?; tail -3 gpurun_out/shard_ab/tests.log; [ $rc -eq 0 ] || exit $rc
rm -f gpurun_out/shard_ab/ab.txt
VARIANTS="${VARIANTS:-build_base build}" REPS=${REPS:-2} bash tools/prof/shard_ab.sh
