#!/bin/bash
# wave multi-read pair counter (sharded path): serial 8-virtual-shard A/B, then the sharded GPU tests
set -u
mkdir -p gpurun_out
for i in 1 2; do
 for v in build_prev build; do
  SA_OVERLAP_LIB=$PWD/sequence-aligner_amd/$v/libsa_overlap.so timeout -k 10 200 python bench.py --shards 8 --serial-shards --steps 3 --warmup 1 --no-cpu-baseline --align-steps 1 > gpurun_out/ab_sh.log 2>&1 || { echo "fail sh $v" >> gpurun_out/ab_pmw.txt; tail -3 gpurun_out/ab_sh.log; exit 1; }
  echo "sh8 $v $(tail -1 gpurun_out/ab_sh.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); s=d["stage_ms_per_step"]; print(d["ms_per_step"], s)')" >> gpurun_out/ab_pmw.txt
 done
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_sharded.py tests/test_gpu_parity.py -m gpu -v --timeout 200 --timeout-method thread -k "shard or rank or multi" > gpurun_out/gpu_tests_sh.log 2>&1; echo "tests rc=$?" >> gpurun_out/ab_pmw.txt
