#!/bin/bash
# Same-box comparison of several source trees on the train bench, interleaved rounds:
# bash tools/ab_dirs.sh <tag> <rounds> <dir> [<dir> ...]   (dirs relative to the repo root; "." = this tree)
set -o pipefail
TAG=$1; R=$2
shift 2
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
mkdir -p gpurun_out
for i in $(seq 1 $R); do
  for D in "$@"; do
    k=$(echo $D | tr -c 'a-zA-Z0-9\n' '_')
    (cd $ROOT/$D && timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-roofline-step) \
      > gpurun_out/${TAG}_${k}_$i.json 2> gpurun_out/${TAG}_${k}_$i.err || { echo "bench failed"; tail -20 gpurun_out/${TAG}_${k}_$i.err; exit 2; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'])" \
      gpurun_out/${TAG}_${k}_$i.json "$D #$i"
  done
done
