#!/bin/bash
# bn3 folded into conv3 for the bf16 scoring forward (VCG_FOLD_BN): tests, then alternating fwd / config-5 benches.
set -o pipefail
TAG=${1:-fold}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_gpu_bf16_train.py::test_eval_bn3_fold_matches_unfolded tests/test_gpu_long_video.py tests/test_gpu_single_modes.py tests/test_gpu_parity.py tests/test_gpu_kernels.py -k "fold or long or single or parity or gemm or c5 or window or mode" > gpurun_out/${TAG}_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/${TAG}_tests.log; exit 1; }
grep -E "vision emb|passed|failed" gpurun_out/${TAG}_tests.log | tail -4
for i in 1 2; do
  for v in 1 0; do
    VCG_FOLD_BN=$v timeout -k 10 300 python bench.py --mode fwd --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/${TAG}_fwd$v$i.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/${TAG}_fwd$v$i.log; exit 1; }
    echo "fwd fold=$v: $(grep -o '"value": [0-9.]*' gpurun_out/${TAG}_fwd$v$i.log)"
  done
done
for v in 1 0; do
  VCG_FOLD_BN=$v timeout -k 10 400 python bench.py --mode long_video > gpurun_out/${TAG}_c5$v.log 2>&1 || { echo "c5 failed"; tail -20 gpurun_out/${TAG}_c5$v.log; exit 1; }
  echo "c5 fold=$v: $(grep -o '"value": [0-9.]*' gpurun_out/${TAG}_c5$v.log) $(grep -o '"f": [0-9.]*' gpurun_out/${TAG}_c5$v.log)"
done
timeout -k 10 600 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/${TAG}_prof -o run -- python bench.py --mode fwd --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/${TAG}_prof.log 2>&1 || { echo "profile failed"; tail -20 gpurun_out/${TAG}_prof.log; exit 3; }
echo done
