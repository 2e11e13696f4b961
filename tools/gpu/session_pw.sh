#!/bin/bash
# wave-per-read pair counter: A/B vs the previous tree, then the GPU tests
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
step smoke 240 python __graft_entry__.py smoke
VARIANTS="build_prev build" REPS=4 step ab_multi 300 bash tools/gpu/ab_multi.sh
step gpu_tests 700 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread
exit 0
