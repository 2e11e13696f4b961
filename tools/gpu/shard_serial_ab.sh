set -u
R=$PWD
timeout -k 10 400 python -u -m pytest tests/test_gpu_sharded.py tests/test_gpu_scale.py -k "shard" -x -q --timeout 300 --timeout-method thread > gpurun_out/t.log 2>&1 || exit 1
for i in 1 2; do for v in abl new; do
  if [ $v = abl ]; then export SA_OVERLAP_LIB=$R/sequence-aligner_amd/build_abl/libsa_overlap.so; else unset SA_OVERLAP_LIB; fi
  timeout -k 10 300 python bench.py --shards 8 --serial-shards --steps 3 --warmup 1 --no-cpu-baseline --align-steps 1 > gpurun_out/sh_${v}_$i.log 2>&1 || exit 1
done; done
