#!/bin/bash
# run-to-run outliers vs the HIP hardware-queue count: the default bench 4x at GPU_MAX_HW_QUEUES=4 (the box
# default) and 4x at 8, interleaved
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for i in 1 2 3 4; do
  for q in 4 8; do
    GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/hwq_${q}_$i.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/hwq_${q}_$i.log; exit 1; }
    echo "q=$q run $i: $(tail -1 gpurun_out/hwq_${q}_$i.log | cut -c100-175)"
  done
done
