#!/bin/bash
# fused BERT attention: its tests + the BERT-touching suites, then a same-box bench A/B (fused vs unfused)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 200 --timeout-method thread tests/test_gpu_bert_attn.py > gpurun_out/attn_tests.log 2>&1 || { echo "attn tests failed"; grep -E "fused|Error|error|assert" gpurun_out/attn_tests.log | tail -30; exit 1; }
grep -E "fused .* unfused|grad rel|passed|failed" gpurun_out/attn_tests.log | tail -30
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_bf16_train.py tests/test_gpu_single_modes.py tests/test_gpu_parity.py > gpurun_out/attn_suites.log 2>&1 || { echo "suites failed"; tail -30 gpurun_out/attn_suites.log; exit 1; }
tail -1 gpurun_out/attn_suites.log
for i in 1 2; do
  VCG_FUSED_ATTN=1 timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/attn_on$i.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/attn_on$i.log; exit 1; }
  echo "fused:   $(tail -1 gpurun_out/attn_on$i.log | cut -c100-200)"
  VCG_FUSED_ATTN=0 timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/attn_off$i.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/attn_off$i.log; exit 1; }
  echo "unfused: $(tail -1 gpurun_out/attn_off$i.log | cut -c100-200)"
done
