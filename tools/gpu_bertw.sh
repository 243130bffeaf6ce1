#!/bin/bash
# BERT's weight gradients on a side stream (BertEncoderEngine.wgrad_stream): the BERT / train-step tests, then the
# same-box train-bench A/B (A = on, B = off).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_bert_attn.py tests/test_gpu_bf16_train.py tests/test_gpu_ddp.py -x -q -rf --timeout 300 --timeout-method thread > gpurun_out/bw_tests.log 2>&1 || { echo tests failed; grep -E "^E |FAILED" gpurun_out/bw_tests.log | head -20; exit 7; }
tail -1 gpurun_out/bw_tests.log
TAG=bertw bash tools/ab_attr.sh vcg_hip.bert.BertEncoderEngine.wgrad_stream=0
