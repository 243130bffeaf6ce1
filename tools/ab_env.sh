#!/bin/bash
# Same-box A/B of one environment flag on the train bench. usage: bash tools/ab_env.sh <tag> <VAR> <A> <B> [rounds]
# [bench args...]  (rounds alternate A, B; each bench under its own time limit)
set -o pipefail
TAG=$1; VAR=$2; VA=$3; VB=$4; R=${5:-2}
shift 5
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for i in $(seq 1 $R); do
  for k in A B; do
    if [ $k = A ]; then V=$VA; else V=$VB; fi
    env "$VAR=$V" timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-roofline-step "$@" \
      > gpurun_out/${TAG}_${k}_$i.json 2> gpurun_out/${TAG}_${k}_$i.err || { echo "bench failed"; tail -20 gpurun_out/${TAG}_${k}_$i.err; exit 2; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'])" \
      gpurun_out/${TAG}_${k}_$i.json "$VAR=$V #$i"
  done
done
