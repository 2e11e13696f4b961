set -u
mkdir -p gpurun_out
timeout -k 10 200 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1 || exit 1
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 10 --warmup 2 > gpurun_out/bench.log 2>&1 || exit 1
bash tools_profile.sh
