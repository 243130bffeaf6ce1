#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_bf16_train.py tests/test_gpu_kernels.py > gpurun_out/bnin_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/bnin_tests.log; exit 1; }
tail -1 gpurun_out/bnin_tests.log
