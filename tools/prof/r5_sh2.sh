set -u
mkdir -p gpurun_out/sh2
timeout -k 10 900 python -u -m pytest tests/test_gpu_sharded.py tests/test_gpu_parity.py tests/test_gpu_big_slices.py -x -v --timeout 600 --timeout-method thread -k "shard or configs3 or rank or sharded" > gpurun_out/sh2/t.log 2>&1
rc=$?; tail -3 gpurun_out/sh2/t.log; [ $rc -eq 0 ] || exit $rc
VARIANTS="build_base build" REPS=2 bash tools/prof/shard_ab.sh
