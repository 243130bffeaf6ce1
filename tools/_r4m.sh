set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_conv_patch.py tests/test_gpu_kernels.py tests/test_gpu_bf16_train.py -m gpu -x -v -k "patch or c1_bf16 or stem" --timeout 200 --timeout-method thread > gpurun_out/r4m_tests.log 2>&1 || { echo "tests failed"; grep -E "PASS|FAIL|Error|error|assert" gpurun_out/r4m_tests.log | tail -40; exit 1; }
grep -E "passed|failed" gpurun_out/r4m_tests.log | tail -3
timeout -k 10 120 python tools/bench_patch.py > gpurun_out/r4m_patch.txt 2>&1; cat gpurun_out/r4m_patch.txt
timeout -k 10 200 python tools/bench_bert_gemm.py > gpurun_out/r4m_bert.txt 2>&1; grep ffn2 gpurun_out/r4m_bert.txt
bash tools/ab_env.sh r4m VCG_FUSED_STEM_BWD 0 1 2
bash tools/gpu_profile.sh r4m
