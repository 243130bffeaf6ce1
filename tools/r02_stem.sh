#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "maxpool or stem or bn" > gpurun_out/stem_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/stem_tests.log; exit 1; }
tail -1 gpurun_out/stem_tests.log
timeout -k 10 200 python -u tools/bench_stem.py 2>&1 | tee gpurun_out/bench_stem.log
