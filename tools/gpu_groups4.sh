#!/bin/bash
# grouped scoring: group streams 3 / 4 / 5 (the caller's + 2 / 3 / 4 extra), fwd and config 5, alternating
set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do for n in 3 4 5; do for m in "--mode fwd --steps 10 --warmup 3" "--mode long_video"; do
  timeout -k 10 300 python bench.py --bn batch --batch 16 --bn-groups 4 --bn-group-streams $n $m --no-cpu-baseline --no-roofline-step > gpurun_out/g4.json 2> gpurun_out/g4.err || { echo "$n $m failed"; tail -20 gpurun_out/g4.err; exit 8; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'])" gpurun_out/g4.json "streams $n $m"
done; done; done
