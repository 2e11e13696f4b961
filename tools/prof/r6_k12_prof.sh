#!/bin/bash
# kernel stats + phase clocks of the configs[4]-shape k = 12 sharded build:
#   tools/prof/r6_k12_prof.sh [reads]   -> gpurun_out/k12prof/
set -u
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/k12prof
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
export SA_DEBUG_PHASES=1
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 \
    $R/tools/prof/r6_k12_2m.py ${1:-1000000} > $OUT/run.log 2> $OUT/phases.log
rc=$?
rm -f $OUT/prof/run_kernel_trace.csv
exit $rc
