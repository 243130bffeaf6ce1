#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_gpu_bert_attn.py tests/test_gpu_bf16_train.py tests/test_gpu_long_video.py -x -q -rfP --timeout 300 --timeout-method thread -k "unpadded or full_res or census or groups or attn" > gpurun_out/cl.log 2>&1; rc=$?
grep -E "passed|failed|unpadded vs|lang_model:|^E " gpurun_out/cl.log | cut -c1-250
[ $rc -eq 0 ] || exit 7
TAG=clslast bash tools/ab_attr.sh vcg_hip.bert.BertEncoderEngine.cls_last=0
