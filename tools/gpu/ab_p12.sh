#!/bin/bash
# A/B of the aligner's phase-1 / phase-2 overlap: build_p12 (split) vs build_nop12
# (-DSA_NO_P12_SPLIT), alternating fresh processes, bench shape
mkdir -p gpurun_out
for i in 1 2 3; do
 for v in build_nop12 build_p12; do
  SA_OVERLAP_LIB=$PWD/sequence-aligner_amd/$v/libsa_overlap.so timeout -k 10 120 python bench.py --steps 6 --warmup 2 --no-cpu-baseline --align-steps 6 > gpurun_out/ab_p12.log 2>&1 || { echo "fail $v"; tail -3 gpurun_out/ab_p12.log; exit 1; }
  echo "$v $(tail -1 gpurun_out/ab_p12.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["ms_per_align_step"], d["align_kernel_ms"])')" >> gpurun_out/ab_p12.txt
 done
done
