#!/bin/bash
# A/B: the sharded pair counter's largest item target (SA_PMW_CAP), bench shape, 8 serial shards,
# alternating fresh processes on one box
set -u
mkdir -p gpurun_out/r6ab
for rep in 1 2; do
  for cap in 128 256 384; do
    SA_PMW_CAP=$cap timeout -k 10 200 python bench.py --shards 8 --serial-shards --steps 6 --warmup 2 --no-cpu-baseline \
        --align-steps 1 --stage-steps 3 > gpurun_out/r6ab/cap_$cap.log 2>&1 || exit 1
    tail -1 gpurun_out/r6ab/cap_$cap.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('cap $cap', d['ms_per_step'], d['stage_ms_per_step'])"
  done
done
