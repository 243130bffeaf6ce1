#!/bin/bash
# Kernel time of the batch-statistics scoring forward: batches of 16 windows (the reference harness) vs one batch of 64
# (the per-group forward's bound), rocprofv3 kernel stats. usage: bash tools/prof_scoring.sh <tag>
set -o pipefail
TAG=${1:-sc}
mkdir -p gpurun_out
export TMPDIR=/tmp
for B in 16 64; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/${TAG}_b$B -o run -- \
    python3 bench.py --mode fwd --bn batch --batch $B --steps 12 --warmup 2 --no-cpu-baseline --no-roofline-step \
    > gpurun_out/${TAG}_b$B.log 2>&1 || { echo "profile B=$B failed"; tail -20 gpurun_out/${TAG}_b$B.log; exit 1; }
  tail -1 gpurun_out/${TAG}_b$B.log | cut -c1-200
done
