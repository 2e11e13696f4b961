#!/bin/bash
# Round 6: which reduce paths the tier tests take -- kernel stats of each case of
# test_virtual_shards_reduce_tiers (the sort shows as reduce_heads_kernel launches)
set -u
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/tierpaths
cd /tmp && export TMPDIR=/tmp
for c in 6000-False 13000-False 6000-True; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/tierpaths/$c -o run -- \
      python3 -m pytest -q -p no:cacheprovider $R/tests/test_gpu_parity.py -m gpu -k "virtual_shards and $c" \
      > $R/gpurun_out/tierpaths/$c.log 2>&1 || exit 1
  rm -f $R/gpurun_out/tierpaths/$c/run_kernel_trace.csv
done
