#!/bin/bash
# Round 6 final tree: the rank-size (2 x 1.25M) and configs[3] real-density (8 x 1.25M, 250 Mbp)
# sharded runs, each with kernel stats + FETCH / WRITE / SQ / LDS PMC passes (traces trimmed).
set -u
SP_TRIM=1 bash tools/prof/slice_prof.sh c3real --reads 1250000 --shards 8 --serial-shards --lean --steps 2 --warmup 1 \
    --align-steps 1 --stage-steps 1 || exit 1
SP_TRIM=1 bash tools/prof/slice_prof.sh rank2 --reads 1250000 --shards 2 --serial-shards --steps 3 --warmup 1 \
    --align-steps 1 --stage-steps 1 || exit 1
tail -14 gpurun_out/steps.txt
