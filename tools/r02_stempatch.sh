#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_conv_patch.py tests/test_gpu_kernels.py -k "stem or patch" > gpurun_out/stemp_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/stemp_tests.log; exit 1; }
tail -1 gpurun_out/stemp_tests.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/stemp_bench.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/stemp_bench.log; exit 1; }
tail -1 gpurun_out/stemp_bench.log | cut -c1-300
bash tools/r02_prof.sh r02stemp
grep -E "7x4/2" gpurun_out/r02stemp_gemm_breakdown.txt
