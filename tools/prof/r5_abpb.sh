rm -f gpurun_out/ab.txt
VARIANTS="build_bpc0 build build_ppb2bpc5" REPS=3 bash tools/prof/ab.sh; cat gpurun_out/ab.txt
