#!/bin/bash
# Scoring lines for both BN semantics and both precisions (configs 2 and 5) plus the CPU-baseline sweep, on one box.
# usage: bash tools/gpu_measure.sh <tag> [tests...]
set -o pipefail
TAG=${1:-m}
shift
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
if [ $# -gt 0 ]; then
  timeout -k 10 600 python -u -m pytest "$@" -v -m gpu --timeout 300 --timeout-method thread -s > gpurun_out/${TAG}_tests.log 2>&1
  rc=$?; grep -E "PASSED|FAILED|ERROR|rel " gpurun_out/${TAG}_tests.log | tail -40
  [ $rc -le 1 ] || exit $rc
fi
run() {  # name, args...
  local n=$1; shift
  timeout -k 10 400 python bench.py "$@" > gpurun_out/${TAG}_$n.json 2> gpurun_out/${TAG}_$n.err || { echo "$n failed"; tail -5 gpurun_out/${TAG}_$n.err; exit 5; }
  echo "$n: $(tail -1 gpurun_out/${TAG}_$n.json | cut -c1-200)"
}
[ "${BENCH:-1}" = 1 ] && {
run fwd_bf16_running --mode fwd --steps 10 --warmup 3
run fwd_bf16_batch16 --mode fwd --bn batch --steps 20 --warmup 3
run fwd_bf16_batch16_groups4 --mode fwd --bn batch --bn-groups 4 --steps 10 --warmup 3
run fwd_fp32_running --mode fwd --precision fp32 --steps 5 --warmup 2
run fwd_fp32_batch16 --mode fwd --precision fp32 --bn batch --steps 10 --warmup 2
run train_fp32_b64 --precision fp32 --steps 3 --warmup 1 --no-cpu-baseline
run c5_bf16_running --mode long_video
run c5_bf16_batch16 --mode long_video --bn batch
run c5_bf16_batch16_groups4 --mode long_video --bn batch --bn-groups 4
run c5_fp32_batch16_stride4 --mode long_video --bn batch --precision fp32 --stride 4
}
[ "${SWEEP:-0}" = 1 ] || exit 0
timeout -k 10 1100 python -u tools/cpu_sweep.py ${SWEEP_WHAT:-all} ${SWEEP_ARGS:-} --out gpurun_out/${TAG}_cpu_sweep.jsonl 2>&1 | tee gpurun_out/${TAG}_cpu_sweep.log || { echo "sweep failed"; tail -5 gpurun_out/${TAG}_cpu_sweep.log; exit 6; }
cat gpurun_out/${TAG}_cpu_sweep.jsonl | cut -c1-220
