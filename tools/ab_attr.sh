#!/bin/bash
# Same-box alternating A/B of a class-attribute switch: A = defaults, B = the given settings; 3 rounds of the train
# bench (20 steps). usage: TAG=name bash tools/ab_attr.sh Module.Class.attr=value [...]
set -o pipefail
mkdir -p gpurun_out
T=${TAG:-abattr}
rm -f gpurun_out/${T}.txt
for r in 1 2 3; do
  for arm in A B; do
    if [ $arm = A ]; then SETS=""; else SETS="$*"; fi
    timeout -k 10 400 python tools/bench_attr.py $SETS -- --steps 20 --warmup 5 --no-cpu-baseline --no-roofline-step ${BENCH_ARGS} > gpurun_out/${T}_${arm}_$r.json 2> gpurun_out/${T}_${arm}_$r.err || { echo "$arm $r failed"; tail -20 gpurun_out/${T}_${arm}_$r.err; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'])" gpurun_out/${T}_${arm}_$r.json "$arm #$r" | tee -a gpurun_out/${T}.txt
  done
done
