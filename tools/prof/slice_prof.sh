#!/bin/bash
# Profile a large single-GPU slice: rocprofv3 kernel stats, then one PMC pass per
# counter group (FETCH_SIZE / WRITE_SIZE / SQ), all on the SAME workload, so the
# summary (tools/pmc_summary.py) is keyed to it.  Usage:
#   tools/prof/slice_prof.sh <name> <bench args...>
# Outputs under gpurun_out/sp_<name>/; stops at the first failure.
set -u
R=$GRAFT_REPO_ROOT
NAME=$1; shift
OUT=$R/gpurun_out/sp_$NAME
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
BENCH="$R/bench.py --no-cpu-baseline $*"
timeout -k 10 400 python3 $BENCH > $OUT/bench.log 2>&1
rc=$?; echo "sp_$NAME bench rc=$rc" >> $R/gpurun_out/steps.txt
[ $rc -eq 0 ] || exit $rc
tail -1 $OUT/bench.log > $OUT/bench.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 $BENCH > $OUT/prof.log 2>&1
rc=$?; echo "sp_$NAME prof rc=$rc" >> $R/gpurun_out/steps.txt
[ $rc -eq 0 ] || exit $rc
pass() {  # pass <name> <counters...>
    local p=$1; shift
    timeout -k 10 400 rocprofv3 --kernel-trace --pmc "$@" --output-format csv -d $OUT/pmc_$p -o pmc -- python3 $BENCH > $OUT/pmc_$p.log 2>&1
    local rc=$?
    echo "sp_$NAME pmc_$p rc=$rc" >> $R/gpurun_out/steps.txt
    [ $rc -eq 0 ] || exit $rc
}
pass fetch FETCH_SIZE
pass write WRITE_SIZE
pass sq SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY
pass lds SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE
# keyed to the workload (bench.py's config.pmc_key): pmc_summary__<key>.csv
KEY=$(python3 -c 'import json,sys; print(json.loads(open(sys.argv[1]).read())["config"]["pmc_key"])' $OUT/bench.json)
python3 $R/tools/pmc_summary.py $OUT $OUT/pmc_summary__$KEY.csv
# (SP_TRIM=1: drop the per-dispatch traces once summarised -- a large multi-shard run's
# traces pass gpurun's 64 MiB copy-back limit)
if [ -n "${SP_TRIM:-}" ]; then
    rm -f $OUT/pmc_*/pmc_kernel_trace.csv $OUT/pmc_*/pmc_counter_collection.csv $OUT/prof/run_kernel_trace.csv
    du -sh $OUT >> $R/gpurun_out/steps.txt
fi
