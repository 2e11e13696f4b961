#!/bin/bash
# Bucket-build timing across fresh processes on one box (round-1 saw per-process
# modes): N bench processes back to back, one JSON line each in gpurun_out/modes.txt.
set -u
mkdir -p gpurun_out
N=${1:-4}
for i in $(seq 1 "$N"); do
    timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --align-steps 2 > gpurun_out/mode_$i.log 2>&1
    rc=$?
    echo "proc_$i rc=$rc $(grep '^{' gpurun_out/mode_$i.log | tail -1)" >> gpurun_out/modes.txt
    [ $rc -eq 0 ] || exit $rc
done
