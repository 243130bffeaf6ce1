bash tools/gpu_profile.sh r03p || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_epilogue.py tests/test_gpu_long_video.py::test_score_windows_streams_identical -q -m gpu --timeout 200 --timeout-method thread 2>&1 | tail -3
for v in 1 0 1 0; do VCG_FAST_GELU=$v timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r03p_bench_fg$v.log 2>&1 || exit 5; echo "fast_gelu=$v $(tail -1 gpurun_out/r03p_bench_fg$v.log | cut -c150-260)"; done
for k in 1 4; do timeout -k 10 300 python bench.py --mode long_video --bn batch --scoring-streams $k --no-cpu-baseline > gpurun_out/r03p_c5_streams$k.json 2>&1 || exit 6; echo "c5 batch16 streams=$k $(tail -1 gpurun_out/r03p_c5_streams$k.json | cut -c90-200)"; done
