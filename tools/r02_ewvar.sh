#!/bin/bash
# streaming-kernel variants (vision_ew.hip SU / GRID_MAX builds) through tools/bench_ew.py, one process per library
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
L=video-chapter-generation_amd/vcg_hip
for v in base su8 su2 g4k g1k; do
  lib=$PWD/$L/libvcg_hip_$v.so; [ $v = base ] && lib=$PWD/$L/libvcg_hip.so
  echo "== $v"
  VCG_LIB_PATH=$lib timeout -k 10 120 python tools/bench_ew.py > gpurun_out/ewvar_$v.log 2>&1 || { echo "failed $v"; tail -5 gpurun_out/ewvar_$v.log; exit 1; }
  cut -c1-200 gpurun_out/ewvar_$v.log
done
