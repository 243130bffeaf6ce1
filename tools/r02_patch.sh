#!/bin/bash
# patch-conv kernel: parity tests, the conv kernel tests, then a profiled bench step
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_conv_patch.py > gpurun_out/patch_tests.log 2>&1 || { echo "patch tests failed"; tail -40 gpurun_out/patch_tests.log; exit 1; }
grep -E "passed|failed" gpurun_out/patch_tests.log | tail -2
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py > gpurun_out/kern_tests.log 2>&1 || { echo "kernel tests failed"; tail -40 gpurun_out/kern_tests.log; exit 1; }
tail -2 gpurun_out/kern_tests.log
bash tools/r02_prof.sh r02patch
