set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_bf16_train.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r4c_tests.log 2>&1 || { echo "tests failed"; grep -E "PASS|FAIL|Error|error|assert" gpurun_out/r4c_tests.log | tail -40; exit 1; }
grep -E "passed|failed|gram stats|vision emb" gpurun_out/r4c_tests.log | tail -8
bash tools/ab_env.sh r4c VCG_GRAM_STATS 0 1 2
