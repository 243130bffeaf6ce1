#!/bin/bash
# per-step times over a long run next to rocm-smi clock / power / temperature samples (outlier diagnosis)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
( for i in $(seq 1 45); do echo "t=$((i*2))s $(rocm-smi --showclocks --showpower --showtemp 2>/dev/null | grep -E 'sclk|mclk|Power|Temperature \(Sensor junction|Temperature \(Sensor memory' | tr -s ' ' | tr '\n' '|')"; sleep 2; done ) > gpurun_out/throttle_smi.log 2>&1 &
SMI=$!
timeout -k 10 200 python tools/step_trace.py 400 > gpurun_out/throttle_steps.log 2>&1; rc=$?
kill $SMI 2>/dev/null
awk '{print $3}' gpurun_out/throttle_steps.log | sort -n | awk '{a[NR]=$1} END {print "steps", NR, "min", a[1], "median", a[int(NR/2)], "p90", a[int(NR*0.9)], "max", a[NR]}'
exit $rc
