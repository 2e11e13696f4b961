#!/bin/bash
# Round 6: the default bench line (as the driver runs it), then tools/prof/profile.sh
# (kernel stats + PMC passes of the default workload).
set -u
mkdir -p gpurun_out/r6fin
timeout -k 10 600 python bench.py > gpurun_out/r6fin/bench_default.log 2>&1 || exit 1
tail -1 gpurun_out/r6fin/bench_default.log > gpurun_out/r6fin/bench_default.json
python3 -c 'import json; d=json.load(open("gpurun_out/r6fin/bench_default.json")); print(d["ms_per_step"], d["value"], d["ms_per_align_step"], d["roofline"]["frac"], d["config0"]["gpu_end_to_end_s"], d["config2_end_to_end"]["total_s"])'
rm -rf gpurun_out/prof gpurun_out/pmc_*
bash tools/prof/profile.sh > gpurun_out/r6fin/profile.log 2>&1 || exit 1
tail -3 gpurun_out/steps.txt
