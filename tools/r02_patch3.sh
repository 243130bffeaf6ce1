#!/bin/bash
# patch conv in the full stack: conv/trunk/parity tests, then bench + rocprof
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_parity.py tests/test_gpu_bf16_train.py tests/test_gpu_single_modes.py > gpurun_out/p3_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/p3_tests.log; exit 1; }
tail -2 gpurun_out/p3_tests.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/p3_bench.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/p3_bench.log; exit 1; }
tail -1 gpurun_out/p3_bench.log | cut -c1-400
bash tools/r02_prof.sh r02flush
