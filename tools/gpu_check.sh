#!/bin/bash
# One GPU-box session: GPU tests -> bench -> rocprofv3 kernel stats (one stream: per-kernel durations are
# unshared and the GEMM log pairs with the trace in order). Stops at the first failure.
# usage: bash tools/gpu_check.sh <tag> [test-selector]
set -o pipefail
TAG=${1:-run}
SEL=${2:-tests/test_gpu_kernels.py tests/test_gpu_parity.py}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest $SEL -q -m gpu -x --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
tail -2 gpurun_out/${TAG}_tests.log
timeout -k 10 600 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/${TAG}_bench.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/${TAG}_bench.log; exit 2; }
tail -1 gpurun_out/${TAG}_bench.log
export TMPDIR=/tmp
rm -f gpurun_out/${TAG}_gemm.log
VCG_GEMM_LOG=gpurun_out/${TAG}_gemm.log timeout -k 10 600 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/${TAG}_prof -o run -- python bench.py --one-stream --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/${TAG}_prof.log 2>&1 || { echo "profile failed"; tail -20 gpurun_out/${TAG}_prof.log; exit 3; }
echo done
