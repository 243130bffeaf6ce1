#!/bin/bash
# kernel trace of the default (multi-stream) bench step: per-stream busy time and the main stream's gaps
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/streams_prof -o run -- python bench.py --steps 3 --warmup 2 --no-cpu-baseline > gpurun_out/streams_prof.log 2>&1 || { echo "profile failed"; tail -20 gpurun_out/streams_prof.log; exit 3; }
tail -1 gpurun_out/streams_prof.log | cut -c1-150
