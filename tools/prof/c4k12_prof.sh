#!/bin/bash
# configs[4]'s k = 12 slice: per-tier item counts (SA_DEBUG_TIERS) and rocprofv3
# kernel stats, packed tier ($1 = 1) or the two-word table ($1 = 0).
set -u
R=$PWD
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
export SA_DEBUG_TIERS=1 SA_PACKED_TIER=$1
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/c4p$1 -o run -- python3 $R/bench.py --no-cpu-baseline --reads 6250000 --len 1000 --min-len 100 --k 12 --steps 1 --warmup 0 --align-steps 1 > $R/gpurun_out/c4p$1.log 2>&1
echo "c4p$1 rc=$?" >> $R/gpurun_out/steps.txt
