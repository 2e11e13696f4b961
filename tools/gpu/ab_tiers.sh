#!/bin/bash
# recount-tier / multi-read insert fast path: configs[4]-shaped 1M mixed k=12 slice and the
# serial 8-virtual-shard bench (multi-read blocks), build_prev vs build
mkdir -p gpurun_out
for i in 1 2; do
 for v in build_prev build; do
  SA_OVERLAP_LIB=$PWD/sequence-aligner_amd/$v/libsa_overlap.so timeout -k 10 200 python bench.py --reads 1000000 --len 1000 --min-len 100 --k 12 --steps 2 --warmup 1 --no-cpu-baseline --align-steps 1 > gpurun_out/ab_k12.log 2>&1 || { echo "fail k12 $v"; tail -3 gpurun_out/ab_k12.log; exit 1; }
  echo "k12 $v $(tail -1 gpurun_out/ab_k12.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); s=d["stage_ms_per_step"]; print(d["ms_per_step"], s)')" >> gpurun_out/ab_tiers.txt
  SA_OVERLAP_LIB=$PWD/sequence-aligner_amd/$v/libsa_overlap.so timeout -k 10 200 python bench.py --shards 8 --serial-shards --steps 3 --warmup 1 --no-cpu-baseline --align-steps 1 > gpurun_out/ab_sh.log 2>&1 || { echo "fail sh $v"; tail -3 gpurun_out/ab_sh.log; exit 1; }
  echo "sh8 $v $(tail -1 gpurun_out/ab_sh.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); s=d["stage_ms_per_step"]; print(d["ms_per_step"], s)')" >> gpurun_out/ab_tiers.txt
 done
done
