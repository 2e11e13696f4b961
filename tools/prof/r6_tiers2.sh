#!/bin/bash
# Round 6: the reduce-tier tests (virtual shards, forced sort) + the sharded / big-slice set,
# then configs[4]-shape k = 12 at 1M (profiled) and 2M
set -u
mkdir -p gpurun_out/r6tiers
timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -k virtual_shards --timeout 150 \
    --timeout-method thread > gpurun_out/r6tiers/tests_virtual.log 2>&1
rc=$?
tail -3 gpurun_out/r6tiers/tests_virtual.log
[ $rc -eq 0 ] || exit $rc
bash tools/prof/r6_tiers.sh 1000000
