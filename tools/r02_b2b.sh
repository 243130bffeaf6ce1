#!/bin/bash
# back-to-back bench processes with rocm-smi clock / power samples (is the second one's slowdown power management?)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
( for i in $(seq 1 60); do echo "t=$i $(rocm-smi --showclocks --showpower 2>/dev/null | grep -E 'sclk|Power \(W\)' | tr -s ' ' | tr '\n' '|')"; sleep 1; done ) > gpurun_out/b2b_smi.log 2>&1 &
SMI=$!
for r in A B C; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/b2b_$r.log 2>&1 || { kill $SMI; exit 1; }
  echo "$r $(date +%s) $(grep -o '"value": [0-9.]*' gpurun_out/b2b_$r.log)"
done
kill $SMI 2>/dev/null
exit 0
