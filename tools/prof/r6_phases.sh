#!/bin/bash
# Round 6: host phase clocks of the sharded build (SA_DEBUG_PHASES), 8 serial virtual shards
set -u
mkdir -p gpurun_out/r6e
SA_DEBUG_PHASES=1 timeout -k 10 300 python bench.py --shards 8 --serial-shards --steps 4 --warmup 1 --no-cpu-baseline --align-steps 1 --stage-steps 1 > gpurun_out/r6e/phases.log 2>&1 || exit 1
grep "sa phases" gpurun_out/r6e/phases.log | tail -3
tail -1 gpurun_out/r6e/phases.log | cut -c1-300
# configs[3]'s density on 8 lean serial shards (10M reads, 250 Mbp): where a build's wall time goes
SA_DEBUG_PHASES=1 timeout -k 10 600 python bench.py --shards 8 --serial-shards --lean --reads 1250000 --steps 2 --warmup 0 --no-cpu-baseline --align-steps 1 --stage-steps 1 > gpurun_out/r6e/phases_c3.log 2>&1 || exit 1
grep "sa phases" gpurun_out/r6e/phases_c3.log | tail -3
tail -1 gpurun_out/r6e/phases_c3.log | cut -c1-600
