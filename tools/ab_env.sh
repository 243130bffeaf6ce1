#!/bin/bash
# Same-box A/B of an environment knob on the train bench: runs tests given in $TESTS first (if any), then
# alternates bench runs with VAR=A / VAR=B. usage: bash tools/ab_env.sh <tag> <VAR> <A> <B> [rounds]
set -o pipefail
TAG=$1; VAR=$2; A=$3; B=$4; R=${5:-2}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -x -v --timeout 240 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 \
    || { echo "tests failed"; tail -40 gpurun_out/${TAG}_tests.log; exit 1; }
  grep -E "passed|failed" gpurun_out/${TAG}_tests.log | tail -3
fi
for i in $(seq 1 $R); do
  for v in $A $B; do
    env $VAR=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-roofline-step \
      > gpurun_out/${TAG}_${v}_$i.json 2> gpurun_out/${TAG}_${v}_$i.err || { echo "bench failed"; tail -20 gpurun_out/${TAG}_${v}_$i.err; exit 2; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'])" \
      gpurun_out/${TAG}_${v}_$i.json "$VAR=$v #$i"
  done
done
