#!/bin/bash
# configs[4]'s k = 12 per-GPU slice under variant libraries and knobs:
#   VARIANTS="dir[:ENV=v[,ENV=v]] ..."  (dirs under sequence-aligner_amd/), one bench line each
# -> gpurun_out/c4ab/<n>.json; summary lines (pairs stage ms, step ms, dispatch hash) in c4ab/ab.txt
set -u
O=gpurun_out/c4ab
mkdir -p $O
i=0
for v in $VARIANTS; do
    dir=${v%%:*}; envs=""
    [ "$dir" != "$v" ] && envs=$(echo "${v#*:}" | tr ',' ' ')
    i=$((i+1))
    env SA_OVERLAP_LIB=$PWD/sequence-aligner_amd/$dir/libsa_overlap.so $envs timeout -k 10 240 python bench.py --no-cpu-baseline \
        --reads 6250000 --len 1000 --min-len 100 --k 12 --steps 1 --warmup 0 --align-steps 0 --dispatch-hash \
        > $O/$i.log 2>&1
    rc=$?
    grep '^{' $O/$i.log | tail -1 > $O/$i.json
    echo "$v rc=$rc $(python3 -c "import json; d=json.load(open('$O/$i.json')); print(d['stage_ms_per_step']['pairs'], d['ms_per_step'], d.get('dispatch_hash'))" 2>/dev/null)" >> $O/ab.txt
    [ $rc -eq 0 ] || exit $rc
done
cat $O/ab.txt
