#!/bin/bash
# End of round at HEAD: the whole -m gpu suite + smoke + bench (tools/gpu_suite.sh), then PMC traffic / MFMA and the
# committed train line with its CPU baseline (tools/gpu_final_a.sh).
set -o pipefail
bash tools/gpu_suite.sh r06e || exit 7
bash tools/gpu_final_a.sh r06h || exit 8
