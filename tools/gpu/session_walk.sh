#!/bin/bash
# phase-2 walk: A/B (tree / no walk (ablation) / interleaved walks), then the GPU tests on the interleaved build
set -u
mkdir -p gpurun_out
VARIANTS="build build_nowalk build_walk2" REPS=3 timeout -k 10 400 bash tools/gpu/ab_multi.sh > gpurun_out/ab.log 2>&1; rc=$?; echo "ab rc=$rc" >> gpurun_out/steps.txt
[ $rc -le 1 ] || exit $rc
SA_OVERLAP_LIB=$PWD/sequence-aligner_amd/build_walk2/libsa_overlap.so timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; echo "gpu_tests rc=$?" >> gpurun_out/steps.txt
