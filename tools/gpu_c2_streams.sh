#!/bin/bash
# C2 running-statistics scoring: one batch of 64 per step vs 2 batches of 64 on 2 HIP streams per step, alternating
set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do for k in 1 2; do
  timeout -k 10 300 python bench.py --mode fwd --scoring-streams $k --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/c2s.json 2> gpurun_out/c2s.err || { echo "$k failed"; tail -20 gpurun_out/c2s.err; exit 8; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('streams', sys.argv[2], d['value'], d['roofline_step']['frac'])" gpurun_out/c2s.json $k
  cp gpurun_out/c2s.json gpurun_out/c2s_$k.json
done; done
