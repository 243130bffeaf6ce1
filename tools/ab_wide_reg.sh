#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
L=video-chapter-generation_amd/vcg_hip
VCG_LIB_PATH=$L/libvcg_w_reg3.so timeout -k 10 300 python -u -m pytest tests/test_gpu_wide.py -x -q --timeout 120 --timeout-method thread > gpurun_out/reg_tests.log 2>&1 || { echo reg3 tests failed; tail -30 gpurun_out/reg_tests.log; exit 1; }
tail -1 gpurun_out/reg_tests.log
for r in 1 2; do for lib in libvcg_hip.so libvcg_w_reg3.so libvcg_w_reg2.so; do
  VCG_LIB_PATH=$L/$lib timeout -k 10 60 python -u tools/bench_wide.py $lib >> gpurun_out/reg_ab.log 2>&1 || exit 2
done; done
grep layer gpurun_out/reg_ab.log
