#!/bin/bash
# Per-kernel time of the train step in two trees on one box (A = abtree/, B = this tree): rocprofv3 kernel stats of a
# short bench run each, side by side (tools/prof_diff.py). usage: bash tools/ab_prof.sh <tag>
set -o pipefail
TAG=$1
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp
for k in A B; do
  if [ $k = A ]; then D=$ROOT/abtree; else D=$ROOT; fi
  (cd $D && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/gpurun_out/${TAG}_$k -o run -- \
    python3 bench.py --steps 6 --warmup 2 --no-cpu-baseline --no-roofline-step) > gpurun_out/${TAG}_$k.log 2>&1 \
    || { echo "profile $k failed"; tail -20 gpurun_out/${TAG}_$k.log; exit 2; }
  tail -1 gpurun_out/${TAG}_$k.log | cut -c1-120
done
python3 tools/prof_diff.py gpurun_out/${TAG}_A/run_kernel_stats.csv gpurun_out/${TAG}_B/run_kernel_stats.csv
