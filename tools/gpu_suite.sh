#!/bin/bash
# The whole -m gpu suite, smoke() and one bench line at HEAD (the driver's round-end checks, rehearsed).
set -o pipefail
mkdir -p gpurun_out
TAG=${1:-suite}
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { echo "tests failed"; grep -E "^E |FAILED" gpurun_out/${TAG}_tests.log | head -20; tail -5 gpurun_out/${TAG}_tests.log; exit 7; }
tail -2 gpurun_out/${TAG}_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/${TAG}_smoke.log; exit 8; }
tail -2 gpurun_out/${TAG}_smoke.log
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { echo "bench failed"; tail -20 gpurun_out/${TAG}_bench.err; exit 9; }
python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('bench', d['value'], d['ms_per_step'], d['roofline']['frac'])" gpurun_out/${TAG}_bench.json
