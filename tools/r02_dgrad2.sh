#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "dgrad" > gpurun_out/dgrad_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/dgrad_tests.log; exit 1; }
tail -1 gpurun_out/dgrad_tests.log
bash tools/r02_dgrad.sh
