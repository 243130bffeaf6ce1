#!/bin/bash
# MFMA utilisation of the bench step from PMC counters: one rocprofv3 pass (counters only) with
# SQ_VALU_MFMA_BUSY_CYCLES (matrix-pipe busy cycles, summed over SIMDs), SQ_BUSY_CYCLES and GRBM_GUI_ACTIVE
# (GPU-busy clocks, summed over the 8 XCDs), then tools/mfma.py writes profiles/mfma_<mode>_<prec>_b<B>.json.
# usage: bash tools/mfma.sh <tag> [mode]
set -o pipefail
TAG=${1:-mfma}
MODE=${2:-train}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
CTRS="SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
timeout -k 10 600 rocprofv3 --pmc $CTRS --output-format csv -d gpurun_out/${TAG}_pmc -o run -- python bench.py --mode $MODE --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/${TAG}_pmc.log 2>&1 || { echo "pmc pass failed"; tail -20 gpurun_out/${TAG}_pmc.log; exit 1; }
python tools/mfma.py gpurun_out/${TAG}_pmc 3 $MODE
