#!/bin/bash
# Train-step profile at HEAD on one box: (1) the benchmarked configuration (side streams on) under rocprofv3 kernel
# trace -> per-kernel stats + GPU idle time (tools/trace_gaps.py); (2) one stream (--one-stream: launch order = start
# order, so the dispatch log pairs with the trace) with the GEMM dispatch log -> time
# per GEMM shape (tools/gemm_breakdown.py). usage: bash tools/gpu_profile.sh <tag> [bench args...]
set -o pipefail
TAG=${1:-prof}
shift
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/${TAG}_trace -o run -- \
  python3 bench.py --steps 4 --warmup 2 --no-cpu-baseline --no-roofline-step "$@" > gpurun_out/${TAG}_trace.log 2>&1 || { echo "trace failed"; tail -20 gpurun_out/${TAG}_trace.log; exit 3; }
tail -1 gpurun_out/${TAG}_trace.log | cut -c1-300
KT=$(find gpurun_out/${TAG}_trace -name "*kernel_trace.csv" | head -1)
ST=$(find gpurun_out/${TAG}_trace -name "*kernel_stats.csv" | head -1)
python3 tools/trace_gaps.py "$KT" --last-ms 300 | tee gpurun_out/${TAG}_gaps.txt
head -25 "$ST" | cut -d, -f1-5
rm -f gpurun_out/${TAG}_gemm.log
VCG_GEMM_LOG=gpurun_out/${TAG}_gemm.log timeout -k 10 600 \
  rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${TAG}_one -o run -- \
  python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --one-stream "$@" > gpurun_out/${TAG}_one.log 2>&1 || { echo "one-stream profile failed"; tail -20 gpurun_out/${TAG}_one.log; exit 4; }
KT1=$(find gpurun_out/${TAG}_one -name "*kernel_trace.csv" | head -1)
python3 tools/gemm_breakdown.py gpurun_out/${TAG}_gemm.log "$KT1" 4 60 > gpurun_out/${TAG}_gemm_breakdown.txt
head -30 gpurun_out/${TAG}_gemm_breakdown.txt
