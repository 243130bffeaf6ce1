#!/bin/bash
# train bench with the synthetic subtitles' padding (default) vs every window's subtitle filling all 128 tokens
set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do for a in "" "--full-text"; do
  timeout -k 10 400 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-roofline-step $a > gpurun_out/ft.json 2> gpurun_out/ft.err || { echo "$a failed"; tail -20 gpurun_out/ft.err; exit 8; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('text_fill', d['config']['text_fill'], d['value'], d['ms_per_step'])" gpurun_out/ft.json
done; done
