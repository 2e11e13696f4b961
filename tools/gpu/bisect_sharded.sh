#!/bin/bash
# which variant library breaks test_sharded_hip_matches_single_gpu[2-True]
mkdir -p gpurun_out
for v in ${VARIANTS:-build_nop12 build_p12 build_bitop build}; do
  SA_OVERLAP_LIB=$PWD/sequence-aligner_amd/$v/libsa_overlap.so timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread "tests/test_gpu_parity.py::test_sharded_hip_matches_single_gpu[2-True]" > gpurun_out/bisect_$v.log 2>&1
  rc=$?
  echo "$v rc=$rc" >> gpurun_out/bisect.txt
  [ $rc -le 1 ] || exit $rc
done
