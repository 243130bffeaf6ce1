#!/bin/bash
# kernel stats + GEMM breakdown of the bench step (one stream: unshared durations)
set -o pipefail
TAG=${1:-r02prof}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -f gpurun_out/${TAG}_gemm.log
VCG_OVERLAP=0 VCG_WGRAD_STREAM=0 VCG_DS_STREAM=0 VCG_PREP_SIDE=0 VCG_GEMM_LOG=gpurun_out/${TAG}_gemm.log timeout -k 10 600 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/${TAG}_prof -o run -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/${TAG}_prof.log 2>&1 || { echo "profile failed"; tail -20 gpurun_out/${TAG}_prof.log; exit 3; }
python tools/gemm_breakdown.py gpurun_out/${TAG}_gemm.log $(ls gpurun_out/${TAG}_prof/*/run_kernel_trace.csv 2>/dev/null || find gpurun_out/${TAG}_prof -name "*kernel_trace.csv" | head -1) 4 60 > gpurun_out/${TAG}_gemm_breakdown.txt
head -3 gpurun_out/${TAG}_gemm_breakdown.txt
echo done
