set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_gpu_bert_attn.py tests/test_gpu_bf16_train.py -x -q -rf --timeout 300 --timeout-method thread -k "attn or varlen or unpadded or full_res" > gpurun_out/at_tests.log 2>&1 || { echo tests failed; grep -E "^E |FAILED" gpurun_out/at_tests.log | head -20; exit 1; }
tail -1 gpurun_out/at_tests.log
TAG=attn bash tools/ab_lib.sh libvcg_w_attnold.so
