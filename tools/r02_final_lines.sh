#!/bin/bash
# Bench lines at HEAD: C2 fwd (scoring, with cpu_baseline), config 5 long video, default train step.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python bench.py --mode fwd > gpurun_out/fl_fwd.log 2>&1 || { echo "fwd failed"; tail -20 gpurun_out/fl_fwd.log; exit 1; }
tail -1 gpurun_out/fl_fwd.log | cut -c1-160
timeout -k 10 400 python bench.py --mode long_video > gpurun_out/fl_c5.log 2>&1 || { echo "c5 failed"; tail -20 gpurun_out/fl_c5.log; exit 1; }
tail -1 gpurun_out/fl_c5.log | cut -c1-160
timeout -k 10 500 python bench.py > gpurun_out/fl_train.log 2>&1 || { echo "train failed"; tail -20 gpurun_out/fl_train.log; exit 1; }
tail -1 gpurun_out/fl_train.log | cut -c1-160
