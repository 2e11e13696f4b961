#!/bin/bash
# Round 6 A/B: the reduce routing's estimate factor (m x ratio x F), F = 0.85 (the tree) vs
# variant libraries built from the same tree with F = 0.7 / 1.0 / 1.2 (ab_lib/, SA_OVERLAP_LIB),
# configs[4]-shape k = 12 at 1M reads on 8 virtual shards
set -u
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/abest
for v in main f70 f100 f120 main; do
  if [ $v = main ]; then unset SA_OVERLAP_LIB; else export SA_OVERLAP_LIB=$R/ab_lib/libsa_$v.so; fi
  SA_DEBUG_PHASES=1 timeout -k 10 300 python $R/tools/prof/r6_k12_2m.py 1000000 > $R/gpurun_out/abest/$v.json \
      2> $R/gpurun_out/abest/$v.phases || exit 1
  mv $R/gpurun_out/abest/$v.json $R/gpurun_out/abest/${v}_$RANDOM.json
done
