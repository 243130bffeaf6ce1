#!/bin/bash
# full GPU suite + smoke + default bench
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/full_tests.log 2>&1 || { echo "gpu tests failed"; tail -40 gpurun_out/full_tests.log; exit 1; }
tail -3 gpurun_out/full_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/full_smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/full_smoke.log; exit 1; }
tail -1 gpurun_out/full_smoke.log
timeout -k 10 400 python bench.py > gpurun_out/full_bench.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/full_bench.log; exit 1; }
tail -1 gpurun_out/full_bench.log | cut -c1-300
