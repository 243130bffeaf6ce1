#!/bin/bash
# End-of-round measurement on one box: the train bench line (with its CPU baseline), PMC traffic + MFMA busy of the
# train step, and the scoring lines for both BN semantics (tools/gpu_measure.sh). usage: bash tools/final_measure.sh <tag>
set -o pipefail
TAG=${1:-fin}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python bench.py > gpurun_out/${TAG}_train.json 2> gpurun_out/${TAG}_train.err || { echo "bench failed"; tail -20 gpurun_out/${TAG}_train.err; exit 1; }
tail -1 gpurun_out/${TAG}_train.json | cut -c1-300
bash tools/traffic.sh ${TAG}_tr > gpurun_out/${TAG}_tr.txt 2>&1 || { echo "traffic failed"; exit 2; }
bash tools/mfma.sh ${TAG}_mf > gpurun_out/${TAG}_mf.txt 2>&1 || { echo "mfma failed"; exit 3; }
bash tools/gpu_measure.sh ${TAG}_m
