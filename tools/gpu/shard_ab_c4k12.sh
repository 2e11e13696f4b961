set -u
timeout -k 10 400 python -u -m pytest tests/test_gpu_sharded.py tests/test_gpu_scale.py -k "shard" -x -q --timeout 300 --timeout-method thread > gpurun_out/t.log 2>&1 || exit 1
for v in base new; do
  L=""; [ $v = base ] && L="SA_OVERLAP_LIB=$PWD/sequence-aligner_amd/build_base/libsa_overlap.so"
  env $L timeout -k 10 300 python bench.py --shards 8 --steps 3 --warmup 1 --no-cpu-baseline --align-steps 1 > gpurun_out/sh_$v.log 2>&1 || exit 1
done
timeout -k 10 900 python -u bench.py --no-cpu-baseline --reads 6250000 --len 1000 --min-len 100 --k 12 --steps 1 --warmup 0 --align-steps 1 > gpurun_out/c4k12.log 2>&1
echo rc=$? >> gpurun_out/c4k12.log
