#!/bin/bash
# Round 6 A/B on one box: the committed library (ab_lib/libsa_old.so, built from HEAD) vs the
# working tree's, configs[3] real density on 8 lean virtual shards, kernel stats each
set -u
R=$GRAFT_REPO_ROOT
for v in old new old new; do
  if [ $v = old ]; then export SA_OVERLAP_LIB=$R/ab_lib/libsa_old.so; else unset SA_OVERLAP_LIB; fi
  bash $R/tools/prof/r6_kstats.sh ab_$v --reads 1250000 --shards 8 --serial-shards --lean --steps 2 --warmup 1 \
      --align-steps 1 --stage-steps 1 || exit 1
  mv $R/gpurun_out/ks_ab_$v $R/gpurun_out/ks_ab_${v}_$RANDOM
done
