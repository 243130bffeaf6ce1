#!/bin/bash
# Same-box alternating train-bench A/B of two builds of libvcg_hip.so (VCG_LIB_PATH): A = the product build, B = the
# named variant (tools/build_variant.sh). usage: TAG=name bash tools/ab_lib.sh libvcg_w_variant.so
set -o pipefail
mkdir -p gpurun_out
T=${TAG:-ablib}
L=video-chapter-generation_amd/vcg_hip
rm -f gpurun_out/${T}.txt
for r in 1 2 3; do
  for arm in A B; do
    LIB=libvcg_hip.so; [ $arm = B ] && LIB=$1
    VCG_LIB_PATH=$L/$LIB timeout -k 10 400 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-roofline-step ${BENCH_ARGS} > gpurun_out/${T}_${arm}_$r.json 2> gpurun_out/${T}_${arm}_$r.err || { echo "$arm $r failed"; tail -20 gpurun_out/${T}_${arm}_$r.err; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'])" gpurun_out/${T}_${arm}_$r.json "$arm #$r" | tee -a gpurun_out/${T}.txt
  done
done
