#!/bin/bash
mkdir -p gpurun_out
for ab in 0 1 2 4 6 7; do
  SA_ABLATE=$ab timeout -k 10 120 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --align-steps 1 > gpurun_out/ab_$ab.log 2>&1 || { echo "ablate $ab failed rc=$?"; exit 1; }
done
