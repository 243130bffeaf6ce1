#!/bin/bash
# BN-on-load (bn2 -> conv3) A/B on one box: kernel tests, then the default bench with and without it, alternating.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_kernels.py -k "bn_on_load or stem or maxpool" > gpurun_out/bnab_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/bnab_tests.log; exit 1; }
tail -1 gpurun_out/bnab_tests.log
for i in 1 2; do
  VCG_BNIN=1 timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bnab_on$i.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bnab_on$i.log; exit 1; }
  echo "on:  $(tail -1 gpurun_out/bnab_on$i.log | cut -c1-120)"
  VCG_BNIN=0 timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bnab_off$i.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bnab_off$i.log; exit 1; }
  echo "off: $(tail -1 gpurun_out/bnab_off$i.log | cut -c1-120)"
done
