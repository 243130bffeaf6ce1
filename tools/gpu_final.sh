#!/bin/bash
# Round-end measurement on one box: full GPU suite, smoke, the train bench line with its CPU baseline.
# usage: bash tools/gpu_final.sh <tag>
set -o pipefail
TAG=${1:-final}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
tail -2 gpurun_out/${TAG}_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/${TAG}_smoke.log; exit 2; }
tail -1 gpurun_out/${TAG}_smoke.log
timeout -k 10 600 python bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { echo "bench failed"; tail -20 gpurun_out/${TAG}_bench.err; exit 3; }
tail -1 gpurun_out/${TAG}_bench.json | cut -c1-400
