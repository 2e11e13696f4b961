#!/bin/bash
# Round 6: directory-gather probe into gpurun_out/r6probe/
set -u
mkdir -p gpurun_out/r6probe
for a in "dir 48600000 30" "dir 607500000 30" "dir 48600000 26" "dir 607500000 28" "span 48600000 389 389" "span 607500000 4860 4860"; do
    timeout -k 10 120 ./tools/scatter_probe $a >> gpurun_out/r6probe/probe.txt 2>&1 || exit $?
done
cat gpurun_out/r6probe/probe.txt
