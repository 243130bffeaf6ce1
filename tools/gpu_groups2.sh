#!/bin/bash
# Per-group scoring: the groups' trunks on 1 / 2 / 4 streams (TwoStream.bn_group_streams), alternating, one box.
set -o pipefail
mkdir -p gpurun_out
T=${TAG:-gr2}
for r in 1 2; do for a in "--batch 16" "--batch 16 --bn-groups 4" "--batch 16 --bn-groups 4 --bn-group-streams 2" "--batch 16 --bn-groups 4 --bn-group-streams 4" "--batch 16 --bn-groups 8 --bn-group-streams 4" "--batch 64"; do
  timeout -k 10 300 python bench.py --mode fwd --bn batch $a --steps 20 --warmup 3 --no-cpu-baseline --no-roofline-step > gpurun_out/${T}_fwd.json 2>gpurun_out/${T}_fwd.err || { echo "fwd $a failed"; tail -20 gpurun_out/${T}_fwd.err; exit 2; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'])" gpurun_out/${T}_fwd.json "$a"
done; done
timeout -k 10 300 python -u -m pytest tests/test_gpu_long_video.py -x -q --timeout 200 --timeout-method thread -k "groups" > gpurun_out/${T}_tests.log 2>&1 || { echo tests failed; tail -30 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log
