#!/bin/bash
# Round 6: the device Trove layout -- strict-id GPU tests, then the default bench (config0 end to end)
set -u
mkdir -p gpurun_out/r6k
OUT=r6k TESTS="tests/test_gpu_parity.py tests/test_gpu_scale.py tests/test_gpu_sharded.py tests/test_cli_modes.py tests/test_afg.py" \
    K="crp177 or ruddii or strict or cli or afg or trove" SECS=600 PER=300 bash tools/prof/r6_tests.sh || exit 1
timeout -k 10 600 python bench.py > gpurun_out/r6k/bench.log 2>&1 || exit 1
tail -1 gpurun_out/r6k/bench.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], json.dumps(d["config0"])[:900])'
