#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_bf16_train.py tests/test_gpu_single_modes.py -m gpu -q -s --timeout 300 --timeout-method thread -rA > gpurun_out/r02b_tests.log 2>&1
echo "tests rc=$?"
grep -E "passed|failed" gpurun_out/r02b_tests.log | tail -3
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r02b_bench_train.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/r02b_bench_train.log; exit 2; }
tail -1 gpurun_out/r02b_bench_train.log
