#!/bin/bash
# Round-5 baseline kernel stats: 8 serial virtual shards of the bench shape, and
# configs[4]'s k = 12 slice with its tier item counts.
set -u
R=$PWD
mkdir -p $R/gpurun_out/r05/base
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r05/base/sh8 -o run -- python3 $R/bench.py --shards 8 --serial-shards --steps 3 --warmup 1 --no-cpu-baseline --align-steps 1 > $R/gpurun_out/r05/base/sh8.log 2>&1 || exit 1
SA_DEBUG_TIERS=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r05/base/c4k12 -o run -- python3 $R/bench.py --no-cpu-baseline --reads 6250000 --len 1000 --min-len 100 --k 12 --steps 1 --warmup 0 --align-steps 1 > $R/gpurun_out/r05/base/c4k12.log 2>&1 || exit 1
