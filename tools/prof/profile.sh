#!/bin/bash
# Kernel statistics and PMC passes over a short bench run (one counter group per
# pass, as MI355X_MICROARCH.md prescribes: FETCH_SIZE and WRITE_SIZE cannot
# share a pass).  Outputs under gpurun_out/; copy the summaries worth keeping
# into profiles/<round>/ (pmc_summary*__<workload>.csv is what bench.py's
# traffic / VALU fields read; the default bench workload is n100000_L500_k15).
set -u
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
BENCH="$R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --align-steps 2"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof -o run -- python3 $BENCH > $R/gpurun_out/prof.log 2>&1
rc=$?
echo "prof rc=$rc" >> $R/gpurun_out/steps.txt
if [ $rc -ne 0 ]; then echo "stopping after prof (rc=$rc)"; exit $rc; fi
pass() {  # pass <name> <counters...>
    local name=$1; shift
    timeout -k 10 300 rocprofv3 --kernel-trace --pmc "$@" --output-format csv -d $R/gpurun_out/pmc_$name -o pmc -- python3 $BENCH > $R/gpurun_out/pmc_$name.log 2>&1
    local rc=$?
    echo "pmc_$name rc=$rc" >> $R/gpurun_out/steps.txt
    if [ $rc -ne 0 ]; then echo "stopping after pmc_$name (rc=$rc)"; exit $rc; fi
}
pass fetch FETCH_SIZE
pass write WRITE_SIZE
pass lds SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE
# the lane-group aligner (LDS traceback, DPP) is not the default at the bench
# shape; one LDS pass over it gives that DP kernel's bank-conflict rate
BENCH="$BENCH --align-kernel 1" pass lds_group SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE
pass clk GRBM_GUI_ACTIVE GRBM_COUNT
pass sq SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY
python3 $R/tools/pmc_summary.py $R/gpurun_out $R/gpurun_out/pmc_summary__n100000_L500_k15.csv
