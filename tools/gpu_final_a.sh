#!/bin/bash
# End-of-round set, part 1 (one box): PMC HBM traffic + MFMA busy of the train step (profiles/traffic_*, mfma_*), then
# the train bench line with its CPU baseline (which reads those files). part 2: tools/gpu_measure.sh (scoring lines).
set -o pipefail
TAG=${1:-r06f}
mkdir -p gpurun_out
bash tools/traffic.sh ${TAG}_tr > gpurun_out/${TAG}_tr.txt 2>&1 || { echo "traffic failed"; tail -20 gpurun_out/${TAG}_tr.txt; exit 2; }
tail -3 gpurun_out/${TAG}_tr.txt
bash tools/mfma.sh ${TAG}_mf > gpurun_out/${TAG}_mf.txt 2>&1 || { echo "mfma failed"; tail -20 gpurun_out/${TAG}_mf.txt; exit 3; }
tail -3 gpurun_out/${TAG}_mf.txt
timeout -k 10 600 python bench.py > gpurun_out/${TAG}_train.json 2> gpurun_out/${TAG}_train.err || { echo "bench failed"; tail -20 gpurun_out/${TAG}_train.err; exit 1; }
python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print('bench', d['value'], d['ms_per_step'], r['frac'], r['traffic'], d['cpu_baseline']['value'], d['roofline_step']['frac'])" gpurun_out/${TAG}_train.json
mkdir -p gpurun_out/prof_out && cp profiles/traffic_train_bf16_b64.json profiles/mfma_train_bf16_b64.json gpurun_out/prof_out/
