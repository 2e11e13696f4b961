#!/bin/bash
# Same-box A/B of library builds (profiling only).  Each variant is a build
# directory under sequence-aligner_amd/ (e.g. `make OUT=build_x EXTRA=-D...`);
# the bench loads it through SA_OVERLAP_LIB.  Variants run alternately REPS
# times; each line of gpurun_out/ab.txt is "<label>_<rep> rc=<rc> <bench JSON>".
#   bash tools_ab.sh 3 build build_nocap
# Stops at the first failure.
set -u
mkdir -p gpurun_out
REPS=$1; shift
LIBDIR=$PWD/sequence-aligner_amd
for rep in $(seq 1 "$REPS"); do
    for v in "$@"; do
        log=gpurun_out/ab_${v}_$rep.log
        SA_OVERLAP_LIB=$LIBDIR/$v/libsa_overlap.so timeout -k 10 300 \
            python bench.py --steps 10 --warmup 2 --no-cpu-baseline --align-steps 2 > "$log" 2>&1
        rc=$?
        echo "${v}_$rep rc=$rc $(grep '^{' "$log" | tail -1)" >> gpurun_out/ab.txt
        [ $rc -eq 0 ] || exit $rc
    done
done
