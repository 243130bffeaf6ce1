#!/bin/bash
# round-2 GPU session 1: full -m gpu suite, bench train + fwd, rocprofv3 counter list, MFMA PMC pass
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 400 --timeout-method thread -rA > gpurun_out/r02d_tests.log 2>&1 ; echo "tests rc=$?"; grep -E "^(FAILED|ERROR)" gpurun_out/r02d_tests.log
tail -3 gpurun_out/r02d_tests.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r02d_bench_train.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/r02d_bench_train.log; exit 2; }
tail -1 gpurun_out/r02d_bench_train.log
timeout -k 10 300 python bench.py --mode fwd --steps 20 --warmup 5 > gpurun_out/r02d_bench_fwd.log 2>&1 || { echo "bench fwd failed"; tail -30 gpurun_out/r02d_bench_fwd.log; exit 3; }
tail -1 gpurun_out/r02d_bench_fwd.log
timeout -k 10 60 rocprofv3 -L > gpurun_out/r02d_counters.txt 2>&1 || echo "counter list failed"
bash tools/mfma.sh r02d_mfma train || exit 4
echo done
