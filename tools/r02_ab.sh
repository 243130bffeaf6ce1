#!/bin/bash
# Same-box A/B of the default library against vcg_hip/libvcg_hip_ab.so (a build with one change reverted):
# kernel + bf16-train tests on the default build, then alternating benches. usage: bash tools/r02_ab.sh <tag> [test -k expr]
set -o pipefail
TAG=${1:-ab}
SEL=${2:-"gemm or conv or dgrad or bn or stem or patch"}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_kernels.py -k "$SEL" > gpurun_out/${TAG}_tests.log 2>&1 || { echo "kernel tests failed"; tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_tests.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_bf16_train.py tests/test_gpu_parity.py > gpurun_out/${TAG}_suite.log 2>&1 || { echo "suite failed"; tail -30 gpurun_out/${TAG}_suite.log; exit 1; }
tail -1 gpurun_out/${TAG}_suite.log
AB=video-chapter-generation_amd/vcg_hip/libvcg_hip_ab.so
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/${TAG}_new$i.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/${TAG}_new$i.log; exit 1; }
  echo "new: $(tail -1 gpurun_out/${TAG}_new$i.log | cut -c100-200)"
  VCG_LIB_PATH=$PWD/$AB timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/${TAG}_old$i.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/${TAG}_old$i.log; exit 1; }
  echo "old: $(tail -1 gpurun_out/${TAG}_old$i.log | cut -c100-200)"
done
rm -f gpurun_out/${TAG}_gemm.log
VCG_OVERLAP=0 VCG_WGRAD_STREAM=0 VCG_DS_STREAM=0 VCG_PREP_SIDE=0 VCG_GEMM_LOG=gpurun_out/${TAG}_gemm.log timeout -k 10 600 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/${TAG}_prof -o run -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/${TAG}_prof.log 2>&1 || { echo "profile failed"; tail -20 gpurun_out/${TAG}_prof.log; exit 3; }
python tools/gemm_breakdown.py gpurun_out/${TAG}_gemm.log gpurun_out/${TAG}_prof/run_kernel_trace.csv 4 60 > gpurun_out/${TAG}_gemm_breakdown.txt
head -8 gpurun_out/${TAG}_gemm_breakdown.txt | cut -c1-130
