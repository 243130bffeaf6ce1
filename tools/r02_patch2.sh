#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_conv_patch.py > gpurun_out/patch_tests.log 2>&1 || { echo "patch tests failed"; tail -40 gpurun_out/patch_tests.log; exit 1; }
tail -1 gpurun_out/patch_tests.log
timeout -k 10 200 python -u tools/bench_patch.py 2>&1 | tee gpurun_out/bench_patch.log
