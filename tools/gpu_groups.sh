#!/bin/bash
# Per-group batch-statistics scoring on one box: the identity tests, then fwd scoring lines (batches of 16: one per
# forward, 4 per forward with per-batch statistics, 4 streams; one batch of 64 = the bound) and config 5.
set -o pipefail
mkdir -p gpurun_out
T=${TAG:-gr}
timeout -k 10 300 python -u -m pytest tests/test_gpu_long_video.py -x -q -rfP --timeout 200 --timeout-method thread -k "groups or streams" > gpurun_out/${T}_tests.log 2>&1 || { echo tests failed; tail -30 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log
for a in "--batch 16" "--batch 16 --bn-groups 4" "--batch 16 --scoring-streams 4" "--batch 64" "--batch 16 --bn-groups 8"; do
  timeout -k 10 300 python bench.py --mode fwd --bn batch $a --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/${T}_fwd.json 2>gpurun_out/${T}_fwd.err || { echo "fwd $a failed"; tail -20 gpurun_out/${T}_fwd.err; exit 2; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d.get('roofline_step',{}).get('frac'))" gpurun_out/${T}_fwd.json "$a"
  cp gpurun_out/${T}_fwd.json "gpurun_out/${T}_fwd_$(echo $a | tr -d ' -').json"
done
for a in "--batch 16" "--batch 16 --bn-groups 4"; do
  timeout -k 10 300 python bench.py --mode long_video --bn batch --stride 4 $a --no-cpu-baseline > gpurun_out/${T}_c5.json 2>gpurun_out/${T}_c5.err || { echo "c5 $a failed"; tail -20 gpurun_out/${T}_c5.err; exit 3; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('c5', sys.argv[2], d['value'], d['boundary']['f'])" gpurun_out/${T}_c5.json "$a"
  cp gpurun_out/${T}_c5.json "gpurun_out/${T}_c5_$(echo $a | tr -d ' -').json"
done
