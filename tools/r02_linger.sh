#!/bin/bash
# what persists between two bench processes: processes on the GPU, memory, clocks; bench -> wait -> bench
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
snap() { echo "--- $1"; rocm-smi --showpids --showmeminfo vram --showclocks 2>/dev/null | grep -E "PID|[0-9]+ +python|VRAM Total Used|sclk|mclk|fclk" | tr -s ' ' | head -12; ps -eo pid,stat,etime,cmd | grep -E "python|bench" | grep -v grep | head; }
snap start
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/linger_1.log 2>&1; echo "run 1 rc $? $(tail -1 gpurun_out/linger_1.log | cut -c100-160)"
snap after1
sleep 20
snap after-sleep
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/linger_2.log 2>&1; echo "run 2 rc $? $(tail -1 gpurun_out/linger_2.log | cut -c100-160)"
timeout -k 10 120 python tools/step_trace.py 20 > gpurun_out/linger_3.log 2>&1; echo "step_trace after: $(awk 'NR>3 {s+=$3; n++} END {printf "%.1f ms", s/n}' gpurun_out/linger_3.log)"
