#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/bench_dgrad.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/bench_dgrad.log
VCG_LIB_PATH=$PWD/video-chapter-generation_amd/build/libvcg_stamps.so timeout -k 10 200 python -u tools/bench_dgrad.py 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/bench_dgrad.log
