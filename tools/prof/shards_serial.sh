#!/bin/bash
# Kernel stats of 8 virtual shards run one after another (SA_OPT_SERIAL_SHARDS):
# per-shard stage times for DESIGN.md 7 (profiles/<round>/sharded/).
set -u
R=$PWD
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/p_sh -o run -- python3 $R/bench.py --shards 8 --serial-shards --steps 3 --warmup 1 --no-cpu-baseline --align-steps 1 > $R/gpurun_out/p_sh.log 2>&1 || exit 1
