#!/bin/bash
# Same-box A/B of an environment switch: kernel tests (-k expr), bf16 train + parity suites, alternating benches.
# usage: bash tools/r02_envab.sh <tag> <VAR> <test -k expr>
set -o pipefail
TAG=$1; VAR=$2; SEL=$3
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_kernels.py -k "$SEL" > gpurun_out/${TAG}_tests.log 2>&1 || { echo "kernel tests failed"; tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_tests.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_bf16_train.py tests/test_gpu_parity.py > gpurun_out/${TAG}_suite.log 2>&1 || { echo "suite failed"; tail -30 gpurun_out/${TAG}_suite.log; exit 1; }
tail -1 gpurun_out/${TAG}_suite.log
for i in 1 2; do
  env $VAR=1 timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/${TAG}_on$i.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/${TAG}_on$i.log; exit 1; }
  echo "on:  $(tail -1 gpurun_out/${TAG}_on$i.log | cut -c100-200)"
  env $VAR=0 timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/${TAG}_off$i.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/${TAG}_off$i.log; exit 1; }
  echo "off: $(tail -1 gpurun_out/${TAG}_off$i.log | cut -c100-200)"
done
