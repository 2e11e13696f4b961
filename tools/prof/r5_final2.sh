#!/bin/bash
# Round-5 final tree: GPU suite, bucket-build stamps, kernel stats + PMC passes, default bench line,
# 8 serial virtual shards, configs[4] k = 12 slice line.  Stops at the first failing step.
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-r05final2}
mkdir -p $O
cd $R
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread --durations=10 > $O/gpu_tests.log 2>&1
rc=$?; echo "gpu_tests rc=$rc" >> $O/steps.txt; tail -3 $O/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
SA_OVERLAP_LIB=$R/sequence-aligner_amd/build_stamps/libsa_overlap.so SA_PB_STAMPS_OUT=$O/stamps.bin \
  timeout -k 10 120 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --align-steps 1 > $O/stamps_bench.log 2>&1
rc=$?; echo "stamps rc=$rc" >> $O/steps.txt; [ $rc -eq 0 ] || exit $rc
python3 tools/pb_stamps.py $O/stamps.bin > $O/pb_stamps.txt 2>&1
bash tools/prof/profile.sh
rc=$?; echo "profile rc=$rc" >> $O/steps.txt; [ $rc -eq 0 ] || exit $rc
cd $R && timeout -k 10 300 python bench.py > $O/bench.log 2>&1
rc=$?; echo "bench rc=$rc" >> $O/steps.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --shards 8 --serial-shards --steps 4 --warmup 1 --no-cpu-baseline --align-steps 1 > $O/sh8.log 2>&1
rc=$?; echo "sh8 rc=$rc" >> $O/steps.txt; [ $rc -eq 0 ] || exit $rc
SA_DEBUG_TIERS=1 timeout -k 10 300 python bench.py --no-cpu-baseline --reads 6250000 --len 1000 --min-len 100 --k 12 --steps 1 --warmup 0 --align-steps 1 --dispatch-hash > $O/c4k12.log 2>&1
rc=$?; echo "c4k12 rc=$rc" >> $O/steps.txt
tail -1 $O/bench.log | cut -c1-300
exit $rc
