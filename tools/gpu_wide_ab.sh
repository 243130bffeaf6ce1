#!/bin/bash
# Wide-tile engine on one box (tools/bench_wide.py): the libraries named in LIBS (default: the product build) in
# alternation, then per-phase stamps (a -DVCG_WIDE_STAMPS build from tools/build_variant.sh). usage: bash tools/gpu_wide_ab.sh
set -o pipefail
mkdir -p gpurun_out
L=video-chapter-generation_amd/vcg_hip
OUT=gpurun_out/${TAG:-w2}.log
for r in 1 2; do for lib in ${LIBS:-libvcg_hip.so}; do
  VCG_LIB_PATH=$L/$lib timeout -k 10 60 python -u tools/bench_wide.py $lib >> $OUT 2>&1 || exit 1
done; done
for n in "768 3072" "3072 768"; do
  echo "stamps N K = $n" >> $OUT
  VCG_LIB_PATH=$L/libvcg_w_stamps.so timeout -k 10 60 python -u tools/wide_stamps.py $n >> $OUT 2>&1 || exit 3
done
