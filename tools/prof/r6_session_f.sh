#!/bin/bash
# Round 6: sharded tests, phase clocks (bench shape, configs[3] density lean), real-density test
set -u
mkdir -p gpurun_out/r6f
OUT=r6f TESTS="tests/test_gpu_sharded.py" SECS=400 PER=300 bash tools/prof/r6_tests.sh || exit 1
SA_DEBUG_PHASES=1 timeout -k 10 300 python bench.py --shards 8 --serial-shards --steps 4 --warmup 1 --no-cpu-baseline --align-steps 1 --stage-steps 1 > gpurun_out/r6f/phases.log 2>&1 || exit 1
grep "sa phases" gpurun_out/r6f/phases.log | tail -2
SA_DEBUG_PHASES=1 timeout -k 10 600 python bench.py --shards 8 --serial-shards --lean --reads 1250000 --steps 3 --warmup 1 --no-cpu-baseline --align-steps 1 --stage-steps 1 > gpurun_out/r6f/phases_c3.log 2>&1 || exit 1
grep "sa phases" gpurun_out/r6f/phases_c3.log | tail -2 | cut -c1-400
tail -1 gpurun_out/r6f/phases_c3.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["stage_ms_per_step"], d["shard_info"], d["first_build_ms"])'
