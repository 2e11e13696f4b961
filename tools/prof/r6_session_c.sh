#!/bin/bash
# Round 6: same-box A/B of the sharded step (round-5 library vs this tree), then the
# default bench line (with the CPU baselines and the end-to-end fields).
set -u
mkdir -p gpurun_out/r6c
VARIANTS="build_r5 build" REPS=3 ARGS="--shards 8 --serial-shards" AB_TIMEOUT=150 bash tools/prof/ab.sh || exit 1
mv gpurun_out/ab.txt gpurun_out/r6c/ab_sharded8.txt
timeout -k 10 600 python bench.py > gpurun_out/r6c/bench.log 2>&1 || exit 1
tail -1 gpurun_out/r6c/bench.log > gpurun_out/r6c/bench.json
cat gpurun_out/r6c/ab_sharded8.txt
