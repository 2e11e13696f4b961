#!/bin/bash
# profiling-only ablation sweep (results are wrong under SA_ABLATE; timing only)
mkdir -p gpurun_out
for ab in 0 1 2 4 6 7 16 32 48; do
  SA_ABLATE=$ab timeout -k 10 120 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --align-steps 1 > gpurun_out/ab_$ab.log 2>&1 || { echo "ablate $ab failed rc=$?"; exit 1; }
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 -L > $GRAFT_REPO_ROOT/gpurun_out/counters.txt 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/pmc1 -o pmc -- python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 0 --no-cpu-baseline --align-steps 1 > $GRAFT_REPO_ROOT/gpurun_out/pmc1.log 2>&1
echo "pmc1 rc=$?"
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/pmc2 -o pmc -- python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 0 --no-cpu-baseline --align-steps 1 > $GRAFT_REPO_ROOT/gpurun_out/pmc2.log 2>&1
echo "pmc2 rc=$?"
