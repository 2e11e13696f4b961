#!/bin/bash
# configs[4]'s k = 12 per-GPU slice under variant libraries ($VARIANTS: build dirs
# under sequence-aligner_amd/), one bench line each -> gpurun_out/c4ab_<dir>.json
set -u
mkdir -p gpurun_out
for v in $VARIANTS; do
    SA_OVERLAP_LIB=$PWD/sequence-aligner_amd/$v/libsa_overlap.so timeout -k 10 420 python bench.py --no-cpu-baseline \
        --reads 6250000 --len 1000 --min-len 100 --k 12 --steps 1 --warmup 0 --align-steps 1 --dispatch-hash \
        > gpurun_out/c4ab_$v.log 2>&1
    rc=$?
    echo "c4ab_$v rc=$rc" >> gpurun_out/steps.txt
    grep '^{' gpurun_out/c4ab_$v.log | tail -1 > gpurun_out/c4ab_$v.json
    [ $rc -eq 0 ] || exit $rc
done
