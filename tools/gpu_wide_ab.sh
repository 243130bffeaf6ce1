#!/bin/bash
# Wide-tile engine A/B on one box (tools/bench_wide.py): pipeline variants in alternation, then per-phase stamps of the
# variants named in STAMP_PIPES (a -DVCG_WIDE_STAMPS build from tools/build_variant.sh). usage: bash tools/gpu_wide_ab.sh
set -o pipefail
mkdir -p gpurun_out
L=video-chapter-generation_amd/vcg_hip
OUT=gpurun_out/${TAG:-w2}.log
for r in 1 2; do for p in ${PIPES:-3 4 13 14 23 24}; do
  VCG_WIDE_PIPE=$p timeout -k 10 60 python -u tools/bench_wide.py pipe$p >> $OUT 2>&1 || exit 1
done; done
for p in ${STAMP_PIPES:-3 24}; do for n in "768 3072" "3072 768"; do
  echo "stamps pipe$p N K = $n" >> $OUT
  VCG_WIDE_PIPE=$p VCG_LIB_PATH=$L/libvcg_w_stamps.so timeout -k 10 60 python -u tools/wide_stamps.py $n >> $OUT 2>&1 || exit 3
done; done
