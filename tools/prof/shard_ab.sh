#!/bin/bash
# Same-box A/B of the sharded path: 8 serial virtual shards of the bench shape
# (bench.py --shards 8 --serial-shards), per-shard stage ms per variant.
#   VARIANTS="dir[:ENV=v[,ENV=v]] ..."  REPS=2  ARGS=extra bench args
set -u
O=gpurun_out/shard_ab
mkdir -p $O
for i in $(seq 1 ${REPS:-2}); do
 for v in $VARIANTS; do
  dir=${v%%:*}; envs=""
  [ "$dir" != "$v" ] && envs=$(echo "${v#*:}" | tr ',' ' ')
  env SA_OVERLAP_LIB=$PWD/sequence-aligner_amd/$dir/libsa_overlap.so $envs timeout -k 10 180 python bench.py --shards 8 --serial-shards --steps 4 --warmup 1 --no-cpu-baseline --align-steps 1 ${ARGS:-} > $O/run.log 2>&1 || { echo "fail $v"; tail -5 $O/run.log; exit 1; }
  echo "$v $(grep '^{' $O/run.log | tail -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); s=d["stage_ms_per_step"]; print(d["ms_per_step"], " ".join("%s=%.3f" % (k, v) for k, v in s.items()))')" | tee -a $O/ab.txt
 done
done
