#!/bin/bash
# the final tree: smoke, every GPU test, the default bench line
set -u
mkdir -p gpurun_out
timeout -k 10 240 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc" >> gpurun_out/steps.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 700 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?; echo "gpu_tests rc=$rc" >> gpurun_out/steps.txt
[ $rc -le 1 ] || exit $rc
timeout -k 10 400 python bench.py > gpurun_out/bench.log 2>&1; echo "bench rc=$?" >> gpurun_out/steps.txt
