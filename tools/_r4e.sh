set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_bnfold.py -m gpu -x -q -k "bn_res_relu" --timeout 120 --timeout-method thread > gpurun_out/r4e_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r4e_tests.log; exit 1; }
tail -2 gpurun_out/r4e_tests.log
timeout -k 10 200 python tools/bench_bnres.py
