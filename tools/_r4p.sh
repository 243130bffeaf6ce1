set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_bnfold.py tests/test_gpu_bf16_train.py -m gpu -x -q -k "stem_bwd_fused or pooled_stem or gram or wgrad or splitk or c1_bf16" --timeout 200 --timeout-method thread > gpurun_out/r4p_tests.log 2>&1 || { echo "tests failed"; grep -E "PASS|FAIL|Error|error|assert" gpurun_out/r4p_tests.log | tail -40; exit 1; }
grep -E "passed|failed" gpurun_out/r4p_tests.log | tail -3
timeout -k 10 120 python tools/bench_stem_bwd.py || exit 1
bash tools/ab_env.sh r4p VCG_SPLITK_WG 1024 512 2
bash tools/ab_env.sh r4p2 VCG_GRAM_STATS 0 1 1
