set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_bf16_train.py tests/test_gpu_torch_ops.py -m gpu -x -v -k "sums_pooled or pooled_stem or linear_op or fused_stem or maxpool_bwd_bn" --timeout 200 --timeout-method thread > gpurun_out/r4l_tests.log 2>&1 || { echo "tests failed"; grep -E "PASS|FAIL|Error|error|assert" gpurun_out/r4l_tests.log | tail -40; exit 1; }
grep -E "passed|failed" gpurun_out/r4l_tests.log | tail -3
bash tools/_r4k.sh || exit 1
bash tools/ab_env.sh r4l VCG_POOLED_STEM_SUMS 0 1 2
