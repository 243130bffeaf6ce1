#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_parity.py tests/test_gpu_bf16_train.py tests/test_gpu_window_train.py tests/test_gpu_single_modes.py > gpurun_out/ew_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/ew_tests.log; exit 1; }
tail -1 gpurun_out/ew_tests.log


timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/ew_bench.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/ew_bench.log; exit 1; }
tail -1 gpurun_out/ew_bench.log | cut -c1-300
bash tools/r02_prof.sh r02bnin
