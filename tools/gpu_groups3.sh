#!/bin/bash
# Committed lines of the per-group scoring: identity tests, fwd batch-statistics line (4 x 16 windows per forward) with
# the roofline step and the CPU baseline, config 5 (stride 4, batches of 16, 4 per forward).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_long_video.py -x -q --timeout 200 --timeout-method thread -k "groups or streams" > gpurun_out/gr3_tests.log 2>&1 || { echo tests failed; tail -30 gpurun_out/gr3_tests.log; exit 1; }
tail -1 gpurun_out/gr3_tests.log
timeout -k 10 400 python bench.py --mode fwd --bn batch --batch 16 --bn-groups 4 --steps 20 --warmup 3 > gpurun_out/gr3_fwd.json 2>gpurun_out/gr3_fwd.err || { echo fwd failed; tail -20 gpurun_out/gr3_fwd.err; exit 2; }
python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('fwd', d['value'], d['ms_per_step'], d['roofline_step']['frac'], d['cpu_baseline']['value'])" gpurun_out/gr3_fwd.json
timeout -k 10 400 python bench.py --mode long_video --bn batch --stride 4 --batch 16 --bn-groups 4 > gpurun_out/gr3_c5.json 2>gpurun_out/gr3_c5.err || { echo c5 failed; tail -20 gpurun_out/gr3_c5.err; exit 3; }
python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('c5', d['value'], d['boundary']['f'])" gpurun_out/gr3_c5.json
