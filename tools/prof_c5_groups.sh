#!/bin/bash
# Kernel trace of config 5 with 4 batch-statistics groups per forward: GPU idle time (tools/trace_gaps.py)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/c5g_trace -o run -- python3 bench.py --mode long_video --bn batch --batch 16 --bn-groups 4 --no-cpu-baseline > gpurun_out/c5g.log 2>&1 || { echo failed; tail -20 gpurun_out/c5g.log; exit 7; }
grep '"metric"' gpurun_out/c5g.log | cut -c1-200
KT=$(find gpurun_out/c5g_trace -name "*kernel_trace.csv" | head -1)
python3 tools/trace_gaps.py "$KT" --last-ms 1500
