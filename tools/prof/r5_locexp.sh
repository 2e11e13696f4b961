#!/bin/bash
# locality experiment: 8 serial virtual shards with each shard's reads in genome order
# (SA_BENCH_SORTED_READS=1: read ids already in locality order), and the single device
set -u
mkdir -p gpurun_out/loc
for v in 0 1; do
  SA_BENCH_SORTED_READS=$v timeout -k 10 200 python bench.py --shards 8 --serial-shards --steps 4 --warmup 1 --no-cpu-baseline --align-steps 1 > gpurun_out/loc/sh8_$v.log 2>&1 || exit 1
  echo "sh8 sorted=$v $(grep '^{' gpurun_out/loc/sh8_$v.log | tail -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["stage_ms_per_step"], d["per_gpu"]["dispatched"])')" | tee -a gpurun_out/loc/ab.txt
done
for v in 0 1; do
  SA_BENCH_SORTED_READS=$v timeout -k 10 200 python bench.py --steps 6 --warmup 2 --no-cpu-baseline --align-steps 1 > gpurun_out/loc/s1_$v.log 2>&1 || exit 1
  echo "single sorted=$v $(tail -1 gpurun_out/loc/s1_$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["stage_ms_per_step"], d["per_gpu"]["dispatched"])')" | tee -a gpurun_out/loc/ab.txt
done
