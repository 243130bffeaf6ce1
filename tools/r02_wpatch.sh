#!/bin/bash
# layer-1 3x3 weight gradient on the LDS patch: kernel tests, the bf16 train suite, bench A/B (VCG_WGRAD_PATCH)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "wgrad" > gpurun_out/wp_tests.log 2>&1 || { echo "kernel tests failed"; grep -E "PASS|FAIL|Error|error|assert" gpurun_out/wp_tests.log | tail -30; exit 1; }
grep -cE "PASSED" gpurun_out/wp_tests.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_bf16_train.py > gpurun_out/wp_suite.log 2>&1 || { echo "bf16 suite failed"; tail -30 gpurun_out/wp_suite.log; exit 1; }
tail -1 gpurun_out/wp_suite.log
for i in 1 2; do
  VCG_WGRAD_PATCH=1 timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/wp_on$i.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/wp_on$i.log; exit 1; }
  echo "patch:  $(tail -1 gpurun_out/wp_on$i.log | cut -c100-200)"
  VCG_WGRAD_PATCH=0 timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/wp_off$i.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/wp_off$i.log; exit 1; }
  echo "im2col: $(tail -1 gpurun_out/wp_off$i.log | cut -c100-200)"
done
rm -f gpurun_out/wp_gemm.log
VCG_OVERLAP=0 VCG_WGRAD_STREAM=0 VCG_GEMM_LOG=gpurun_out/wp_gemm.log timeout -k 10 600 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/wp_prof -o run -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/wp_prof.log 2>&1 || { echo "profile failed"; tail -20 gpurun_out/wp_prof.log; exit 3; }
grep -E "wgrad3x3|wgrad_fast|splitk" gpurun_out/wp_prof/run_kernel_stats.csv | cut -d, -f1-4
