#!/bin/bash
# Round-5 final-tree measurement: bucket-build block stamps (timing-probe build),
# kernel stats + PMC passes (profile.sh), then the default bench line.
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05final
mkdir -p $O
cd $R
SA_OVERLAP_LIB=$R/sequence-aligner_amd/build_stamps/libsa_overlap.so SA_PB_STAMPS_OUT=$O/stamps.bin \
  timeout -k 10 120 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --align-steps 1 > $O/stamps_bench.log 2>&1
rc=$?; echo "stamps rc=$rc" >> $O/steps.txt; [ $rc -eq 0 ] || exit $rc
python3 tools/pb_stamps.py $O/stamps.bin > $O/pb_stamps.txt 2>&1
bash tools/prof/profile.sh
rc=$?; echo "profile rc=$rc" >> $O/steps.txt; [ $rc -eq 0 ] || exit $rc
cd $R && timeout -k 10 300 python bench.py > $O/bench.log 2>&1
rc=$?; echo "bench rc=$rc" >> $O/steps.txt
tail -1 $O/bench.log | cut -c1-400
exit $rc
