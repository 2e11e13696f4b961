rm -f gpurun_out/ab.txt
VARIANTS="build build:SA_OCC_PW=6 build:SA_OCC_PW=5 build:SA_OCC_SPLIT=4 build:SA_OCC_SPLIT=2 build:SA_OCC_RS=1" REPS=2 bash tools/prof/ab.sh; cat gpurun_out/ab.txt
