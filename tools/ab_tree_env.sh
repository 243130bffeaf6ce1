#!/bin/bash
# Same-box A/B of two source trees (A = abtree/, B = this tree) under one extra environment setting each round:
# bash tools/ab_tree_env.sh <tag> <rounds> "<VAR=value ...>" ["<VAR=value ...>" ...] (each setting runs on A then B)
set -o pipefail
TAG=$1; R=$2
shift 2
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
mkdir -p gpurun_out
for i in $(seq 1 $R); do
  j=0
  for E in "$@"; do
    j=$((j + 1))
    [ "$E" = "-" ] && E=""
    for k in A B; do
      if [ $k = A ]; then D=$ROOT/abtree; else D=$ROOT; fi
      (cd $D && env $E timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-roofline-step) \
        > gpurun_out/${TAG}_${k}${j}_$i.json 2> gpurun_out/${TAG}_${k}${j}_$i.err || { echo "bench failed"; tail -20 gpurun_out/${TAG}_${k}${j}_$i.err; exit 2; }
      python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'])" \
        gpurun_out/${TAG}_${k}${j}_$i.json "$k [$E] #$i"
    done
  done
done
