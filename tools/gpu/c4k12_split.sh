set -u
timeout -k 10 400 python -u -m pytest tests/test_gpu_scale.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline --reads 1000000 --len 1000 --min-len 100 --k 12 --steps 2 --warmup 1 --align-steps 1 > gpurun_out/k12_1m.log 2>&1 || exit 1
bash tools_slice_prof.sh c4k12 --reads 6250000 --len 1000 --min-len 100 --k 12 --steps 1 --warmup 0 --align-steps 1 || exit 1
