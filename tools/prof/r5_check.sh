#!/bin/bash
# GPU suite (all tests) + configs[4] k = 12 slice bench line; stops at the first crash / timeout.
set -u
O=gpurun_out/r05/${TAG:-check}
mkdir -p $O
export SA_TEST_RECORD_DIR=$O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread --durations=15 > $O/gpu_tests.log 2>&1
rc=$?; echo "gpu_tests rc=$rc" >> $O/steps.txt; tail -25 $O/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
SA_DEBUG_TIERS=1 timeout -k 10 300 python bench.py --no-cpu-baseline --reads 6250000 --len 1000 --min-len 100 --k 12 --steps 1 --warmup 0 --align-steps 1 --dispatch-hash > $O/c4k12.log 2>&1
rc=$?; echo "c4k12 rc=$rc" >> $O/steps.txt; grep "sa tiers" $O/c4k12.log | tail -4
tail -1 $O/c4k12.log | cut -c1-600
exit $rc
