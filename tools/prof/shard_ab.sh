#!/bin/bash
# Sharded-path tests, then 8 serial virtual shards of the bench shape under the
# variants in $VARIANTS ("dir[:ENV=v,...]" as tools/prof/ab.sh), alternating;
# one bench line each -> gpurun_out/shab_<n>_<i>.json
set -u
mkdir -p gpurun_out
if [ "${SKIP_TESTS:-0}" != 1 ]; then
timeout -k 10 600 python -u -m pytest tests/test_gpu_sharded.py tests/test_gpu_parity.py tests/test_gpu_scale.py -x -v \
    --timeout 300 --timeout-method thread -k "shard" > gpurun_out/t_shard.log 2>&1
echo "tests rc=$?" >> gpurun_out/steps.txt
fi
for i in 1 2; do
  n=0
  for v in $VARIANTS; do
    n=$((n + 1))
    dir=${v%%:*}; envs="X=1"
    [ "$dir" != "$v" ] && envs=$(echo "${v#*:}" | tr ',' ' ')
    env SA_OVERLAP_LIB=$PWD/sequence-aligner_amd/$dir/libsa_overlap.so $envs timeout -k 10 200 python bench.py \
        --no-cpu-baseline --shards 8 --serial-shards --steps 3 --warmup 1 --align-steps 1 > gpurun_out/shab_${n}_$i.log 2>&1 \
        || { echo "shab $v rc=$?" >> gpurun_out/steps.txt; exit 1; }
    echo "$v $(grep '^{' gpurun_out/shab_${n}_$i.log | tail -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); s=d["stage_ms_per_step"]; print(d["ms_per_step"], s["emit"], s["sort"], s["buckets"], s["pairs"], s["order"])')" >> gpurun_out/shab.txt
  done
done
echo "shab rc=0" >> gpurun_out/steps.txt
