#!/bin/bash
# kernel stats: 8 serial virtual shards of the bench shape, and the single device
set -u
R=$PWD
O=$R/gpurun_out/r05/shprof
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/sh8 -o run -- python3 $R/bench.py --shards 8 --serial-shards --steps 3 --warmup 1 --no-cpu-baseline --align-steps 1 > $O/sh8.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/s1 -o run -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline --align-steps 2 > $O/s1.log 2>&1 || exit 1
