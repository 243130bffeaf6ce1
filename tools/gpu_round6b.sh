#!/bin/bash
# Packing cache per base tensor (long-video batches are slices of one mask): tests, config-5 batch-statistics lines,
# then the BERT side-stream priority A/B (TwoStream.side_priority = -1 vs 0).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_bert_attn.py tests/test_gpu_long_video.py -x -q -rf --timeout 300 --timeout-method thread > gpurun_out/r6b_tests.log 2>&1 || { echo tests failed; grep -E "^E |FAILED" gpurun_out/r6b_tests.log | head -20; exit 7; }
tail -1 gpurun_out/r6b_tests.log
for a in "--bn batch --batch 16" "--bn batch --batch 16 --bn-groups 4" "--bn running"; do
  timeout -k 10 300 python bench.py --mode long_video $a --no-cpu-baseline > gpurun_out/r6b_c5.json 2> gpurun_out/r6b_c5.err || { echo "c5 $a failed"; tail -20 gpurun_out/r6b_c5.err; exit 8; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('c5', sys.argv[2], d['value'], d['roofline_step']['frac'])" gpurun_out/r6b_c5.json "$a"
  cp gpurun_out/r6b_c5.json "gpurun_out/r6b_c5_$(echo $a | tr -d ' -').json"
done
TAG=prio bash tools/ab_attr.sh model.fusion.two_stream.TwoStream.side_priority=-1
