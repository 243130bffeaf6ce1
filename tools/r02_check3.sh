#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_bf16_train.py tests/test_gpu_long_video.py tests/test_gpu_single_modes.py -m gpu -q -s --timeout 600 --timeout-method thread -rA > gpurun_out/r02e_tests.log 2>&1
echo "tests rc=$?"
grep -E "^(PASSED|FAILED|ERROR)|^C5|vision_emb rel|grad rel err vs exact|^loss exact|grad error ratio" gpurun_out/r02e_tests.log
