#!/bin/bash
# rocprofv3 kernel stats of one bench invocation (traces dropped after the summary):
#   tools/prof/r6_kstats.sh <name> <bench args...>   -> gpurun_out/ks_<name>/
set -u
R=$GRAFT_REPO_ROOT
NAME=$1; shift
OUT=$R/gpurun_out/ks_$NAME
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 $R/bench.py \
    --no-cpu-baseline "$@" > $OUT/prof.log 2>&1
rc=$?
rm -f $OUT/prof/run_kernel_trace.csv
tail -1 $OUT/prof.log > $OUT/bench.json
exit $rc
