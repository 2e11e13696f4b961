#!/bin/bash
# GPU tests of the tree, then the 2-rank repeat-case sharded test 5 more times (a flake seen once)
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
step gpu_tests 700 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread
for i in 1 2 3 4 5; do
  step rep_$i 200 python -u -m pytest -x -q --timeout 150 --timeout-method thread "tests/test_gpu_parity.py::test_sharded_hip_matches_single_gpu[2-True]"
done
exit 0
