#!/bin/bash
# full GPU suite, then kernel stats of the sharded path (8 serial virtual shards)
set -u
O=gpurun_out/r05/${TAG:-suite}
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread --durations=10 > $O/gpu_tests.log 2>&1
rc=$?; echo "gpu_tests rc=$rc" >> $O/steps.txt; tail -14 $O/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
bash tools/prof/r5_shprof.sh
