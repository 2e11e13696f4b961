#!/bin/bash
# same-box A/B: base library (build_base) vs the tree's, plus any extra build
# directories named in $AB_EXTRA (e.g. "build_v1 build_v2"), alternating
mkdir -p gpurun_out
for i in 1 2 3; do
 for v in base new ${AB_EXTRA:-}; do
  case $v in
   base) L="SA_OVERLAP_LIB=$PWD/sequence-aligner_amd/build_base/libsa_overlap.so" ;;
   new) L="" ;;
   *) L="SA_OVERLAP_LIB=$PWD/sequence-aligner_amd/$v/libsa_overlap.so" ;;
  esac
  env $L timeout -k 10 120 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --align-steps 4 > gpurun_out/ab.log 2>&1 || { echo fail; tail -3 gpurun_out/ab.log; exit 1; }
  echo "$v $(tail -1 gpurun_out/ab.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); s=d["stage_ms_per_step"]; print(d["ms_per_step"], s["sort"], s["buckets"], s["pairs"], d["ms_per_align_step"], d["align_kernel_ms"])')" >> gpurun_out/ab.txt
 done
done
