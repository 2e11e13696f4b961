#!/bin/bash
# Round 6: the lead-reduce tiers -- the sharded / repeat / big-slice GPU tests, then the
# configs[4]-shape k = 12 profile (tools/prof/r6_k12_prof.sh)
set -u
mkdir -p gpurun_out/r6tiers
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_big_slices.py -m gpu -x -v \
    -k "shard or repeat or k12 or dist" --timeout 300 --timeout-method thread > gpurun_out/r6tiers/tests.log 2>&1
rc=$?
tail -3 gpurun_out/r6tiers/tests.log
[ $rc -eq 0 ] || exit $rc
bash tools/prof/r6_k12_prof.sh ${1:-1000000}
rc=$?
[ $rc -eq 0 ] || exit $rc
SA_DEBUG_PHASES=1 timeout -k 10 300 python tools/prof/r6_k12_2m.py 2000000 > gpurun_out/r6tiers/k12_2M.json \
    2> gpurun_out/r6tiers/k12_2M_phases.log
