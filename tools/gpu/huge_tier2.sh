set -u
timeout -k 10 500 python -u -m pytest tests/test_gpu_scale.py -x -q --timeout 300 --timeout-method thread -k "recount or per_read or mixed" > gpurun_out/t.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline --reads 1000000 --len 1000 --min-len 100 --k 12 --steps 2 --warmup 1 --align-steps 1 > gpurun_out/k12_1m.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline --reads 1000000 --len 1000 --min-len 100 --k 15 --steps 2 --warmup 1 --align-steps 1 > gpurun_out/k15_1m.log 2>&1 || exit 1
