# build-only timings of the tree's library and ablation builds ($ABL dirs)
mkdir -p gpurun_out
for i in 1 2; do
 for v in build ${ABL:-}; do
  echo "$v $(SA_OVERLAP_LIB=$PWD/sequence-aligner_amd/$v/libsa_overlap.so timeout -k 10 120 python tools/gpu/build_only.py ${ABL_ARGS:-})" >> gpurun_out/abl.txt || exit 1
 done
done
