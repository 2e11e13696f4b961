#!/bin/bash
# smoke + configs[3] per-GPU slice (1.25M x 500 bp, k = 15) on the tree with the block-major radix histograms
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc" >> gpurun_out/steps.txt; [ $rc -eq 0 ] || exit $rc
bash tools_slices.sh c3
