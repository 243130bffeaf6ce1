set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q -k "register_stream or bwd_stream_vs" --timeout 120 --timeout-method thread > gpurun_out/r4i_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r4i_tests.log; exit 1; }
tail -2 gpurun_out/r4i_tests.log
for f in 1 0; do VCG_RS_DGRAD=$f VCG_BENCH_NOY=1 timeout -k 10 120 python tools/bench_dgrad.py "" 1 | sed "s/^/RS_DGRAD=$f /" || exit 1; done
