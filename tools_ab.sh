#!/bin/bash
# Same-box A/B of bench variants selected by env (profiling only): each line of
# gpurun_out/ab.txt is "<label> rc=<rc> <bench JSON>".  Stops at the first failure.
#   bash tools_ab.sh occ   bucket-build LDS occupancy (SA_PB_LDS pads)
#   bash tools_ab.sh pc    pair-count compile variants (build_* trees via SA_OVERLAP_LIB)
#   bash tools_ab.sh nt    non-temporal record stores in the bucket build (build_nt: -DSA_REC_NT=1)
#   bash tools_ab.sh pcnt  non-temporal record loads in the pair count (build_pcnt: -DSA_PC_RECNT=1)
#   bash tools_ab.sh sknt  non-temporal sorted-record loads in the bucket build (build_sknt: -DSA_PB_SKNT=1)
#   bash tools_ab.sh listnt non-temporal partner-list stores in the bucket build (build_listnt: -DSA_PB_LISTNT=1)
#   bash tools_ab.sh sk3   current build vs build_sknt vs build_nosknt (-DSA_PB_SKNT=0)
#   bash tools_ab.sh rsknt non-temporal key loads in the radix scatter (build_rsknt: -DSA_RS_KNT=1)
#   bash tools_ab.sh rsvnt non-temporal value loads in the radix scatter (build_rsvnt: -DSA_RS_VNT=1)
#   bash tools_ab.sh rsunt non-temporal key loads in the radix histogram (build_rsunt: -DSA_RS_UNT=1)
#   bash tools_ab.sh contig physically contiguous large buffers (env SA_ALLOC_CONTIG=1), 4 alternations
set -u
mkdir -p gpurun_out
run() {  # run <label> [VAR=value ...]
    local label=$1; shift
    env "$@" timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --align-steps 2 > gpurun_out/ab_$label.log 2>&1
    local rc=$?
    echo "$label rc=$rc $(grep '^{' gpurun_out/ab_$label.log | tail -1)" >> gpurun_out/ab.txt
    [ $rc -eq 0 ] || exit $rc
}
LIBDIR=$PWD/sequence-aligner_amd
case "${1:-occ}" in
occ)
    run occ8_a
    run occ6_a SA_PB_LDS=24704
    run occ8_b
    run occ6_b SA_PB_LDS=24704
    run occ7 SA_PB_LDS=21000
    ;;
pc)
    run base_a
    run batch16 SA_OVERLAP_LIB=$LIBDIR/build_b16/libsa_overlap.so
    run batch4 SA_OVERLAP_LIB=$LIBDIR/build_b4/libsa_overlap.so
    run threads512 SA_OVERLAP_LIB=$LIBDIR/build_t512/libsa_overlap.so
    run base_b
    ;;
nt)
    run base_a
    run nt_a SA_OVERLAP_LIB=$LIBDIR/build_nt/libsa_overlap.so
    run base_b
    run nt_b SA_OVERLAP_LIB=$LIBDIR/build_nt/libsa_overlap.so
    ;;
pcnt)
    run base_a
    run pcnt_a SA_OVERLAP_LIB=$LIBDIR/build_pcnt/libsa_overlap.so
    run base_b
    run pcnt_b SA_OVERLAP_LIB=$LIBDIR/build_pcnt/libsa_overlap.so
    ;;
sknt)
    run base_a
    run sknt_a SA_OVERLAP_LIB=$LIBDIR/build_sknt/libsa_overlap.so
    run base_b
    run sknt_b SA_OVERLAP_LIB=$LIBDIR/build_sknt/libsa_overlap.so
    ;;
listnt)
    run base_a
    run listnt_a SA_OVERLAP_LIB=$LIBDIR/build_listnt/libsa_overlap.so
    run base_b
    run listnt_b SA_OVERLAP_LIB=$LIBDIR/build_listnt/libsa_overlap.so
    ;;
sk3)
    run base_a
    run sknt_a SA_OVERLAP_LIB=$LIBDIR/build_sknt/libsa_overlap.so
    run nosknt_a SA_OVERLAP_LIB=$LIBDIR/build_nosknt/libsa_overlap.so
    run base_b
    run sknt_b SA_OVERLAP_LIB=$LIBDIR/build_sknt/libsa_overlap.so
    run nosknt_b SA_OVERLAP_LIB=$LIBDIR/build_nosknt/libsa_overlap.so
    ;;
rsknt)
    run base_a
    run rsknt_a SA_OVERLAP_LIB=$LIBDIR/build_rsknt/libsa_overlap.so
    run base_b
    run rsknt_b SA_OVERLAP_LIB=$LIBDIR/build_rsknt/libsa_overlap.so
    ;;
rsvnt)
    run base_a
    run rsvnt_a SA_OVERLAP_LIB=$LIBDIR/build_rsvnt/libsa_overlap.so
    run base_b
    run rsvnt_b SA_OVERLAP_LIB=$LIBDIR/build_rsvnt/libsa_overlap.so
    ;;
rsunt)
    run base_a
    run rsunt_a SA_OVERLAP_LIB=$LIBDIR/build_rsunt/libsa_overlap.so
    run base_b
    run rsunt_b SA_OVERLAP_LIB=$LIBDIR/build_rsunt/libsa_overlap.so
    ;;
contig)
    for i in 1 2 3 4; do run base_$i; run contig_$i SA_ALLOC_CONTIG=1; done
    ;;
esac
