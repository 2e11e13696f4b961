VARIANTS="build build:SA_NO_LOCALITY=1" REPS=2 bash tools/prof/ab.sh; cat gpurun_out/ab.txt
