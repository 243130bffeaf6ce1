#!/bin/bash
# Round-2 measurement refresh at HEAD: PMC HBM traffic (FETCH / WRITE passes) and MFMA-busy pass -> profiles/,
# rocprofv3 kernel stats + GEMM breakdown (one stream), then the default bench line and the fwd-only (C2) line.
set -o pipefail
TAG=${1:-r02final}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/traffic.sh ${TAG}_traffic train || exit 1
bash tools/mfma.sh ${TAG}_mfma train || exit 1
bash tools/r02_prof.sh ${TAG} || exit 1
timeout -k 10 400 python bench.py > gpurun_out/${TAG}_bench.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/${TAG}_bench.log; exit 1; }
tail -1 gpurun_out/${TAG}_bench.log | cut -c1-200
timeout -k 10 400 python bench.py --mode fwd > gpurun_out/${TAG}_bench_fwd.log 2>&1 || { echo "fwd bench failed"; tail -20 gpurun_out/${TAG}_bench_fwd.log; exit 1; }
tail -1 gpurun_out/${TAG}_bench_fwd.log | cut -c1-200
cp profiles/traffic_train_bf16_b64.json profiles/mfma_train_bf16_b64.json gpurun_out/
