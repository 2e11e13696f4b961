#!/bin/bash
set -u
mkdir -p gpurun_out
VARIANTS="build build_ntl" REPS=4 timeout -k 10 400 bash tools/gpu/ab_multi.sh > gpurun_out/ab.log 2>&1; echo "ab rc=$?" >> gpurun_out/steps.txt
