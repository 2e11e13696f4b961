#!/bin/bash
# configs[3]'s per-GPU slice (1.25M x 500 bp) on one device: bucket-build blocks per CU 5 vs the register limit
set -u
mkdir -p gpurun_out/c3pb
rm -f gpurun_out/c3pb/ab.txt
for i in 1 2; do
 for v in build build_pb7; do
  SA_OVERLAP_LIB=$PWD/sequence-aligner_amd/$v/libsa_overlap.so timeout -k 10 300 python bench.py --reads 1250000 --steps 3 --warmup 1 --no-cpu-baseline --align-steps 1 > gpurun_out/c3pb/run.log 2>&1 || { echo "fail $v"; tail -3 gpurun_out/c3pb/run.log; exit 1; }
  echo "$v $(tail -1 gpurun_out/c3pb/run.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); s=d["stage_ms_per_step"]; print(d["ms_per_step"], " ".join("%s=%.2f" % (k, v) for k, v in s.items()))')" | tee -a gpurun_out/c3pb/ab.txt
 done
done
