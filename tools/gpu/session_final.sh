#!/bin/bash
# final evidence of a tree: rocprofv3 kernel stats + PMC passes (tools_profile.sh), the PMC summary
# placed under profiles/$VER/ so the bench line that follows cites it, then the default bench line
set -u
mkdir -p gpurun_out
VER=${VER:-r03/v3}
bash tools_profile.sh || exit $?
mkdir -p profiles/$VER
cp gpurun_out/pmc_summary__n100000_L500_k15.csv profiles/$VER/ || exit 1
timeout -k 10 400 python bench.py > gpurun_out/bench_final.log 2>&1
rc=$?; echo "bench_final rc=$rc" >> gpurun_out/steps.txt
exit $rc
