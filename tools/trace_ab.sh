#!/bin/bash
# Kernel traces of the train bench for two values of an environment knob, with per-queue busy time and kernel
# stats. usage: bash tools/trace_ab.sh <tag> <VAR> <A> <B>
set -o pipefail
TAG=$1; VAR=$2
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in $3 $4; do
  D=gpurun_out/${TAG}_${v}
  env $VAR=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $D -o run -- \
    python3 bench.py --steps 4 --warmup 2 --no-cpu-baseline --no-roofline-step > $D.log 2>&1 || { echo "trace failed"; tail -20 $D.log; exit 3; }
  tail -1 $D.log | cut -c1-200
  KT=$(find $D -name "*kernel_trace.csv" | head -1)
  ST=$(find $D -name "*kernel_stats.csv" | head -1)
  python3 tools/queue_busy.py "$KT" --last-ms 250 --steps 3 > $D.queues.txt
  cp "$ST" $D.stats.csv
  echo "== $VAR=$v"; head -14 $D.queues.txt
done
