#!/bin/bash
# the same workload in 4 consecutive processes: per-step wall / CPU time and host load (run-to-run outliers)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for i in 1 2 3 4; do
  timeout -k 10 120 python tools/step_trace.py 30 > gpurun_out/runs_$i.log 2>&1 || exit 1
  echo "run $i: $(awk 'NR>3 {s+=$3; c+=$11; n++} END {printf "wall %.1f ms cpu %.1f ms", s/n, c/n}' gpurun_out/runs_$i.log) $(tail -1 gpurun_out/runs_$i.log | grep -o 'load.*') nproc $(nproc)"
done
