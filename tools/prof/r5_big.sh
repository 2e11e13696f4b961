set -o pipefail
export SA_TEST_RECORD_DIR=gpurun_out/r05/big
mkdir -p $SA_TEST_RECORD_DIR
timeout -k 10 1000 python -u -m pytest tests/test_gpu_big_slices.py -x -v -s --timeout 900 --timeout-method thread --durations=0 > gpurun_out/r05/big/pytest.log 2>&1
rc=$?; echo "rc=$rc"; tail -30 gpurun_out/r05/big/pytest.log; exit $rc
