#!/bin/bash
# Round-4 slice runs: configs[3]'s per-GPU slice, configs[4]'s k = 12 slice with the
# packed and the two-word recount tier, 8 serial virtual shards with per-read
# regions and with multi-read blocks.  One bench line each under gpurun_out/sl_*.json.
set -u
mkdir -p gpurun_out
run() {  # run <name> <seconds> <env...> -- <bench args...>
    local name=$1 secs=$2; shift 2
    local envs=()
    while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
    env "${envs[@]}" timeout -k 10 "$secs" python bench.py --no-cpu-baseline "$@" > gpurun_out/sl_$name.log 2>&1
    local rc=$?
    echo "sl_$name rc=$rc" >> gpurun_out/steps.txt
    grep '^{' gpurun_out/sl_$name.log | tail -1 > gpurun_out/sl_$name.json
    [ $rc -eq 0 ] || exit $rc
}
run c3 300 X=1 -- --reads 1250000 --steps 3 --warmup 1 --align-steps 1
run sh8 200 X=1 -- --shards 8 --serial-shards --steps 3 --warmup 1 --align-steps 1
run sh8multi 200 SA_SHARD_MULTI=1 -- --shards 8 --serial-shards --steps 3 --warmup 1 --align-steps 1
run c4k12 400 X=1 -- --reads 6250000 --len 1000 --min-len 100 --k 12 --steps 1 --warmup 0 --align-steps 1 --dispatch-hash
run c4k12two 400 SA_PACKED_TIER=0 -- --reads 6250000 --len 1000 --min-len 100 --k 12 --steps 1 --warmup 0 --align-steps 1 --dispatch-hash
