#!/bin/bash
# FETCH_SIZE / WRITE_SIZE per launch of the fused 1x1 dgrads (streaming vs persistent), one rocprofv3 pass per
# counter (MI355X_MICROARCH.md: FETCH_SIZE reads half the bytes of wide streaming reads). usage: bash tools/pmc_dgrad.sh <tag> [shape]
set -o pipefail
TAG=${1:-pmcd}
SHAPE=${2:-l1}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for F in 1 0; do
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 120 rocprofv3 --pmc $C --output-format csv -d gpurun_out/${TAG}_${F}_$C -o run -- python3 tools/bench_dgrad.py $SHAPE $F > gpurun_out/${TAG}_${F}_$C.log 2>&1 || { echo "pmc $C failed"; tail -5 gpurun_out/${TAG}_${F}_$C.log; exit 1; }
    echo "VCG_BWD_STREAM=$F $C: $(python3 tools/pmc_kernel.py gpurun_out/${TAG}_${F}_$C igemm_fast_kernel | head -3)"
  done
done
