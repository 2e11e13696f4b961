#!/bin/bash
# A/B: radix tiles of 2,048 keys (build_t2048) vs 4,096 (build), both with block-major tile histograms
set -u
mkdir -p gpurun_out
VARIANTS="build build_t2048" REPS=4 timeout -k 10 400 bash tools/gpu/ab_multi.sh > gpurun_out/ab.log 2>&1; echo "ab rc=$?" >> gpurun_out/steps.txt
