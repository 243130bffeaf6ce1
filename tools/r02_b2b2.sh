#!/bin/bash
# correctness suites, then 4 back-to-back bench processes with the host / allocator diagnostics
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_bf16_train.py tests/test_gpu_ddp.py tests/test_gpu_parity.py > gpurun_out/b2b2_suite.log 2>&1 || { echo "suite failed"; tail -30 gpurun_out/b2b2_suite.log; exit 1; }
tail -1 gpurun_out/b2b2_suite.log
for r in A B C D; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/b2b2_$r.log 2>&1 || exit 1
  python -c "import json; d=json.loads(open('gpurun_out/b2b2_$r.log').read().strip().splitlines()[-1]); print('$r', d['value'], d['host'])"
done
