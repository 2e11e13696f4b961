#!/bin/bash
# Round 6 A/B: the lead-reduce tier routing (distinct-per-partial ratio vs the m / ranks
# floor alone) at configs[3] real density and configs[4]-shape k = 12, kernel stats each
set -u
R=$GRAFT_REPO_ROOT
for mode in 1 0; do
  export SA_LR_ROUTE=$mode
  bash $R/tools/prof/r6_kstats.sh c3route$mode --reads 1250000 --shards 8 --serial-shards --lean --steps 2 --warmup 1 \
      --align-steps 1 --stage-steps 1 || exit 1
done
