#!/bin/bash
# One GPU-box session at HEAD: the whole -m gpu suite -> the bench line -> tools/gpu_profile.sh (kernel stats of the
# benchmarked configuration + the one-stream GEMM breakdown). Stops at the first failure.
# usage: bash tools/gpu_round.sh <tag> [test selector]
set -o pipefail
TAG=${1:-round}
SEL=${2:-tests}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest $SEL -m gpu -x -q -rfP --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/${TAG}_tests.log; exit 1; }
tail -2 gpurun_out/${TAG}_tests.log
timeout -k 10 600 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { echo "bench failed"; tail -30 gpurun_out/${TAG}_bench.err; exit 2; }
python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('bench', d['value'], d['ms_per_step'], d['roofline']['frac'])" gpurun_out/${TAG}_bench.json
bash tools/gpu_profile.sh ${TAG}p
