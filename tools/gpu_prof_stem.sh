#!/bin/bash
# The round's step profile at HEAD (tools/gpu_profile.sh: concurrent trace + the one-stream GEMM breakdown), then the
# stem backward's parameters-in-registers change against the previous kernel (libvcg_w_stemold.so), alternating.
set -o pipefail
mkdir -p gpurun_out
bash tools/gpu_profile.sh r06c || exit 1
L=video-chapter-generation_amd/vcg_hip
for r in 1 2 3; do for lib in libvcg_hip.so libvcg_w_stemold.so; do
  echo "[$lib]" >> gpurun_out/stem_ab.log
  VCG_LIB_PATH=$L/$lib timeout -k 10 120 python -u tools/bench_stem_bwd.py >> gpurun_out/stem_ab.log 2>&1 || exit 2
done; done
grep -E "^\[|fused" gpurun_out/stem_ab.log
