#!/bin/bash
# smoke + GPU tests + bench + aligner A/B + profile passes, stopping at the first crash / timeout
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
step gpu_tests 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread
step ab_p12 400 bash tools/gpu/ab_p12.sh
step bench 300 python bench.py --steps 10 --warmup 2
[ "${PROF:-1}" = 1 ] && bash tools_profile.sh
exit 0
