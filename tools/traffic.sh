#!/bin/bash
# HBM traffic of the bench step from PMC counters (MI355X_MICROARCH.md § HBM): two separate rocprofv3
# passes (FETCH_SIZE and WRITE_SIZE do not fit one pass), counters only, then tools/traffic.py
# writes profiles/traffic_<mode>_<prec>_b<B>.json. usage: bash tools/traffic.sh <tag> [mode]
set -o pipefail
TAG=${1:-traffic}
MODE=${2:-train}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 900 rocprofv3 --pmc $C --output-format csv -d gpurun_out/${TAG}_$C -o run -- python bench.py --mode $MODE --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/${TAG}_$C.log 2>&1 || { echo "pmc $C failed"; tail -20 gpurun_out/${TAG}_$C.log; exit 1; }
done
python tools/traffic.py gpurun_out/${TAG}_FETCH_SIZE gpurun_out/${TAG}_WRITE_SIZE 3 $MODE
