set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_epilogue.py tests/test_gpu_kernels.py tests/test_gpu_bert_attn.py -m gpu -x -q -k "ffn_gelu or gemm or bert" --timeout 200 --timeout-method thread > gpurun_out/r4u_tests.log 2>&1 || { echo "tests failed"; grep -E "PASS|FAIL|Error|error|assert" gpurun_out/r4u_tests.log | tail -40; exit 1; }
grep -E "passed|failed" gpurun_out/r4u_tests.log | tail -3
bash tools/_r4t.sh
