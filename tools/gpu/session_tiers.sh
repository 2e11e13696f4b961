#!/bin/bash
set -u
mkdir -p gpurun_out
timeout -k 10 900 bash tools/gpu/ab_tiers.sh > gpurun_out/ab_tiers.log 2>&1; rc=$?; echo "ab_tiers rc=$rc" >> gpurun_out/steps.txt
[ $rc -le 1 ] || exit $rc
true
