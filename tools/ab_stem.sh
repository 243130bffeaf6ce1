# A/B of the pair-packed stem (default) against the C = 8 stem (VCG_NO_STEM_PAIR=1), after its tests.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -q -m gpu -x --timeout 300 --timeout-method thread -k "stem_pair or window_frames or conv_fwd or conv_wgrad" > gpurun_out/stem_tests.log 2>&1 || { echo "kernel tests failed"; tail -30 gpurun_out/stem_tests.log; exit 1; }
tail -1 gpurun_out/stem_tests.log
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_long_video.py -q -m gpu -x --timeout 300 --timeout-method thread > gpurun_out/stem_parity.log 2>&1 || { echo "parity tests failed"; tail -30 gpurun_out/stem_parity.log; exit 1; }
tail -1 gpurun_out/stem_parity.log
for i in 1 2; do
  VCG_NO_STEM_PAIR=1 timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/stem_a$i.log 2>&1 || exit 2
  python -c "import json;d=json.loads(open('gpurun_out/stem_a$i.log').read().strip().splitlines()[-1]);print('c8',d['value'],d['ms_per_step'])"
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/stem_c$i.log 2>&1 || exit 2
  python -c "import json;d=json.loads(open('gpurun_out/stem_c$i.log').read().strip().splitlines()[-1]);print('pair',d['value'],d['ms_per_step'])"
done
