#!/bin/bash
# One GPU session: smoke + GPU tests, bench, profile (tools/prof/session.sh [all|tests|bench|prof],
# from the repository root).  Stops at the first crash / timeout.
set -u
mkdir -p gpurun_out
step() {  # step <name> <seconds> <cmd...>
    local name=$1 secs=$2; shift 2
    timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc" >> gpurun_out/steps.txt
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
    return 0
}
MODE=${1:-all}
if [ "$MODE" = all ] || [ "$MODE" = tests ]; then
    step smoke 240 python __graft_entry__.py smoke
    step gpu_tests 1050 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread
fi
if [ "$MODE" = all ] || [ "$MODE" = bench ]; then
    step bench 600 python bench.py --steps 10 --warmup 2
fi
if [ "$MODE" = all ] || [ "$MODE" = prof ]; then
    bash tools/prof/profile.sh
fi
