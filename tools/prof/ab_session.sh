#!/bin/bash
# Tests, then a same-box A/B of the variants in $VARIANTS (tools/prof/ab.sh);
# stops at the first crash / timeout.  Run from the repository root.
set -u
mkdir -p gpurun_out
if [ "${SKIP_TESTS:-0}" != 1 ]; then
    bash tools/prof/session.sh tests
    rc=$?; [ $rc -eq 0 ] || exit $rc
    grep -q "rc=0" gpurun_out/steps.txt || true
fi
timeout -k 10 ${AB_TOTAL:-600} bash tools/prof/ab.sh > gpurun_out/ab_session.log 2>&1
echo "ab rc=$?" >> gpurun_out/steps.txt
