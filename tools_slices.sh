#!/bin/bash
# Large single-GPU slices of BASELINE.json's multi-GPU configs (evidence runs):
#   configs[3] per-GPU slice: 1.25M x 500 bp reads, k = 15
#   configs[4]-shaped slices: mixed 100-1,000 bp reads, k = 15 and k = 12
# One bench line each into gpurun_out/slice_*.json; stops at the first failure.
set -u
mkdir -p gpurun_out
run() {  # run <name> <seconds> <bench args...>
    local name=$1 secs=$2; shift 2
    timeout -k 10 "$secs" python bench.py --no-cpu-baseline "$@" > gpurun_out/slice_$name.log 2>&1
    local rc=$?
    echo "slice_$name rc=$rc" >> gpurun_out/steps.txt
    tail -1 gpurun_out/slice_$name.log > gpurun_out/slice_$name.json
    if [ $rc -ne 0 ]; then echo "stopping after slice_$name (rc=$rc)"; exit $rc; fi
}
SLICES=${1:-all}
if [ "$SLICES" = all ] || [ "$SLICES" = c3 ]; then
    run c3_1250k 300 --reads 1250000 --steps 3 --warmup 1 --align-steps 2
fi
if [ "$SLICES" = all ] || [ "$SLICES" = c4 ]; then
    run c4_1m_k15 300 --reads 1000000 --len 1000 --min-len 100 --k 15 --steps 3 --warmup 1 --align-steps 1
    run c4_1m_k12 300 --reads 1000000 --len 1000 --min-len 100 --k 12 --steps 2 --warmup 1 --align-steps 1
fi
# configs[4]'s full per-GPU slice (50M / 8 = 6.25M mixed reads, ~3.35e9 k-mers:
# the combined partner list runs past 2^32 entries, and the reads past the
# (read, pos) codes' 2^22); then 3M mixed reads (1.6e9 k-mers, list indices past
# 2^32) rebuilt over 4 virtual shards (each under 2^32) must give the identical
# dispatch -- the whole-device sharded context of the 6.25M set does not fit
if [ "$SLICES" = all ] || [ "$SLICES" = c4full ]; then
    run c4_6250k_k15 600 --reads 6250000 --len 1000 --min-len 100 --k 15 --steps 2 --warmup 1 --align-steps 1
    run c4_3m_k15_check 600 --reads 3000000 --len 1000 --min-len 100 --k 15 --steps 2 --warmup 1 --align-steps 1 \
        --check-shards 4
fi
