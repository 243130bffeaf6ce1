#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_window_train.py tests/test_gpu_window.py -m gpu -q -s --timeout 300 --timeout-method thread -rA > gpurun_out/r02f_tests.log 2>&1
echo "tests rc=$?"
grep -E "^(PASSED|FAILED|ERROR)|loss ours|worst grad|bf16 |directional|^E  " gpurun_out/r02f_tests.log | head -60
