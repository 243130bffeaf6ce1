#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_bf16_train.py tests/test_gpu_single_modes.py tests/test_gpu_ddp.py -m gpu -q -s --timeout 400 --timeout-method thread -rA > gpurun_out/r02c_tests.log 2>&1
echo "tests rc=$?"
grep -E "^(PASSED|FAILED|ERROR)" gpurun_out/r02c_tests.log
