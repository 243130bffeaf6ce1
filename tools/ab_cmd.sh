#!/bin/bash
# Same-box A/B of two environment settings on the train bench: bash tools/ab_cmd.sh <tag> "<env A>" "<env B>" [rounds]
# (each setting is a space-separated list of VAR=value, "-" for none)
set -o pipefail
TAG=$1; A=$2; B=$3; R=${4:-2}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for i in $(seq 1 $R); do
  for k in A B; do
    if [ $k = A ]; then E=$A; else E=$B; fi
    [ "$E" = "-" ] && E=""
    env $E timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-roofline-step \
      > gpurun_out/${TAG}_${k}_$i.json 2> gpurun_out/${TAG}_${k}_$i.err || { echo "bench failed"; tail -20 gpurun_out/${TAG}_${k}_$i.err; exit 2; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'])" \
      gpurun_out/${TAG}_${k}_$i.json "$k [$E] #$i"
  done
done
