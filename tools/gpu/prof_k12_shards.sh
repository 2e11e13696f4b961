set -u
R=$PWD
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/p_k12 -o run -- python3 $R/bench.py --no-cpu-baseline --reads 1000000 --len 1000 --min-len 100 --k 12 --steps 1 --warmup 0 --align-steps 1 > $R/gpurun_out/p_k12.log 2>&1 || exit 1
for v in base new; do
  if [ $v = base ]; then export SA_OVERLAP_LIB=$R/sequence-aligner_amd/build_base/libsa_overlap.so; else unset SA_OVERLAP_LIB; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/p_sh_$v -o run -- python3 $R/bench.py --shards 8 --steps 3 --warmup 1 --no-cpu-baseline --align-steps 1 > $R/gpurun_out/p_sh_$v.log 2>&1 || exit 1
done
