#!/bin/bash
# weight gradients on a side stream: the bf16 train / DDP suites, then a same-box bench A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_bf16_train.py tests/test_gpu_ddp.py tests/test_gpu_drivers.py > gpurun_out/ws_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/ws_tests.log; exit 1; }
tail -1 gpurun_out/ws_tests.log
for i in 1 2; do
  VCG_WGRAD_STREAM=1 timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/ws_on$i.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/ws_on$i.log; exit 1; }
  echo "side:   $(tail -1 gpurun_out/ws_on$i.log | cut -c100-200)"
  VCG_WGRAD_STREAM=0 timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/ws_off$i.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/ws_off$i.log; exit 1; }
  echo "single: $(tail -1 gpurun_out/ws_off$i.log | cut -c100-200)"
done
