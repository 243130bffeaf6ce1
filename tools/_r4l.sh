set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_bf16_train.py tests/test_gpu_torch_ops.py tests/test_gpu_epilogue.py -m gpu -x -v -k "linear_op or ffn_gelu" --timeout 200 --timeout-method thread > gpurun_out/r4l_tests.log 2>&1 || { echo "tests failed"; grep -E "PASS|FAIL|Error|error|assert" gpurun_out/r4l_tests.log | tail -40; exit 1; }
grep -E "passed|failed" gpurun_out/r4l_tests.log | tail -3
timeout -k 10 120 python tools/bench_patch.py > gpurun_out/r4l_patch.txt 2>&1; cat gpurun_out/r4l_patch.txt
timeout -k 10 200 python tools/bench_bert_gemm.py > gpurun_out/r4l_bert.txt 2>&1; tail -20 gpurun_out/r4l_bert.txt
bash tools/_r4k.sh || exit 1
bash tools/ab_env.sh r4l VCG_FUSED_STEM_BWD 0 1 2
bash tools/gpu_profile.sh r4l
