#!/bin/bash
# same-box A/B over variant library builds (fresh process each, alternating):
# VARIANTS="build_x build_y ..." (dirs under sequence-aligner_amd/), REPS rounds,
# bench shape; one line per run: variant, hash step, sort, buckets, pairs, align step, align kernel
mkdir -p gpurun_out
for i in $(seq 1 ${REPS:-3}); do
 for v in $VARIANTS; do
  SA_OVERLAP_LIB=$PWD/sequence-aligner_amd/$v/libsa_overlap.so timeout -k 10 120 python bench.py --steps 8 --warmup 2 --no-cpu-baseline --align-steps 6 > gpurun_out/ab_multi.log 2>&1 || { echo "fail $v"; tail -3 gpurun_out/ab_multi.log; exit 1; }
  echo "$v $(tail -1 gpurun_out/ab_multi.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); s=d["stage_ms_per_step"]; print(d["ms_per_step"], s["sort"], s["buckets"], s["pairs"], d["ms_per_align_step"], d["align_kernel_ms"])')" >> gpurun_out/ab_multi.txt
 done
done
