#!/bin/bash
# Round 6: timing check after a change to the sharded reduce -- configs[3] real density on
# 8 lean virtual shards, the rank-size 2-shard run, and the default bench line
set -u
mkdir -p gpurun_out/r6reg
timeout -k 10 300 python bench.py --no-cpu-baseline --reads 1250000 --shards 8 --serial-shards --lean --steps 2 \
    --warmup 1 --align-steps 1 --stage-steps 1 > gpurun_out/r6reg/c3real.log 2>&1 || exit 1
tail -1 gpurun_out/r6reg/c3real.log > gpurun_out/r6reg/c3real.json
timeout -k 10 300 python bench.py --no-cpu-baseline --reads 1250000 --shards 2 --serial-shards --steps 3 --warmup 1 \
    --align-steps 1 --stage-steps 1 > gpurun_out/r6reg/rank2.log 2>&1 || exit 1
tail -1 gpurun_out/r6reg/rank2.log > gpurun_out/r6reg/rank2.json
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/r6reg/default.log 2>&1 || exit 1
tail -1 gpurun_out/r6reg/default.log > gpurun_out/r6reg/default.json
