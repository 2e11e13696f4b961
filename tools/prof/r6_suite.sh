#!/bin/bash
# Round 6: the whole GPU suite (records of the big-slice tests kept) and smoke().
set -u
mkdir -p gpurun_out/r6suite
SA_TEST_RECORD_DIR=gpurun_out/r6suite/rec timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 400 \
    --timeout-method thread > gpurun_out/r6suite/gpu_tests.log 2>&1
rc=$?
tail -3 gpurun_out/r6suite/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r6suite/smoke.log 2>&1
rc=$?
tail -2 gpurun_out/r6suite/smoke.log
exit $rc
