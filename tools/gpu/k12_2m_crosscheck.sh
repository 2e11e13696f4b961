set -u
# 2M mixed reads at k = 12 (reads up to ~25k partners: the residue-class
# tiers): this tree vs the morning's library (256-thread tiers, fixed 1/8/64
# classes -- no wrap at this size), dispatch checksum and counts
for v in abl new; do
  if [ $v = abl ]; then export SA_OVERLAP_LIB=$PWD/sequence-aligner_amd/build_abl/libsa_overlap.so; else unset SA_OVERLAP_LIB; fi
  timeout -k 10 500 python bench.py --no-cpu-baseline --reads 2000000 --len 1000 --min-len 100 --k 12 --steps 1 --warmup 0 --align-steps 1 --dispatch-hash > gpurun_out/x2m_$v.log 2>&1 || exit 1
done
