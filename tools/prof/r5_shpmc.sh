#!/bin/bash
# PMC passes over the sharded path (8 serial virtual shards of the bench shape), one counter group per pass
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/shpmc
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
BENCH="$R/bench.py --shards 8 --serial-shards --steps 2 --warmup 1 --no-cpu-baseline --align-steps 1"
pass() {  # pass <name> <counters...>
    local name=$1; shift
    timeout -k 10 300 rocprofv3 --kernel-trace --pmc "$@" --output-format csv -d $O/pmc_$name -o pmc -- python3 $BENCH > $O/pmc_$name.log 2>&1
    local rc=$?
    echo "pmc_$name rc=$rc" >> $O/steps.txt
    if [ $rc -ne 0 ]; then echo "stopping after pmc_$name (rc=$rc)"; exit $rc; fi
}
pass fetch FETCH_SIZE
pass write WRITE_SIZE
pass lds SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE
pass clk GRBM_GUI_ACTIVE GRBM_COUNT
pass sq SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY
python3 $R/tools/pmc_summary.py $O $O/pmc_summary__sharded8_n100000_L500_k15.csv
