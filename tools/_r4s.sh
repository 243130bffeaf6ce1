set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_conv_patch.py tests/test_gpu_kernels.py -m gpu -x -q -k "patch" --timeout 200 --timeout-method thread > gpurun_out/r4s_tests.log 2>&1 || { echo "tests failed"; grep -E "PASS|FAIL|Error|error|assert" gpurun_out/r4s_tests.log | tail -40; exit 1; }
grep -E "passed|failed" gpurun_out/r4s_tests.log | tail -3
timeout -k 10 120 python tools/bench_patch.py 2>&1 | grep -v amdgpu.ids
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/r4s_fwd -o run -- python3 bench.py --mode fwd --steps 5 --warmup 2 --no-cpu-baseline --no-roofline-step > gpurun_out/r4s_fwd.log 2>&1 || { echo "fwd trace failed"; tail -5 gpurun_out/r4s_fwd.log; exit 3; }
tail -1 gpurun_out/r4s_fwd.log | cut -c1-200
ST=$(find gpurun_out/r4s_fwd -name "*kernel_stats.csv" | head -1)
head -25 "$ST" | cut -d, -f1-5
