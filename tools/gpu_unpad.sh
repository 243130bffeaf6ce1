#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_bert_attn.py tests/test_gpu_bf16_train.py tests/test_gpu_long_video.py -x -q -rfP --timeout 300 --timeout-method thread -k "attn or varlen or unpadded or full_res or census or groups or streams" > gpurun_out/up_tests.log 2>&1 || { echo tests failed; grep -E "Error|error|assert|FAILED" gpurun_out/up_tests.log | head -30; tail -30 gpurun_out/up_tests.log; exit 1; }
tail -1 gpurun_out/up_tests.log
grep -E "lang_model:|unpadded vs padded" gpurun_out/up_tests.log | cut -c1-300
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/up_bench.json 2> gpurun_out/up_bench.err || { echo bench failed; tail -30 gpurun_out/up_bench.err; exit 2; }
python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('bench', d['value'], d['ms_per_step'], d['roofline']['frac'])" gpurun_out/up_bench.json
