#!/bin/bash
# PMC passes (one counter group per rocprofv3 run) over the wide-tile engine on one BERT shape (tools/bench_wide.py
# --only <shape>): L2 hit / miss, memory-side fetch, LDS bank conflicts and busy cycles, MFMA busy.
# usage: bash tools/pmc_wide.sh <shape prefix, e.g. "ffn2 fwd"> [tag]
set -o pipefail
SH=${1:-ffn2 fwd}; TAG=${2:-pmcw}
mkdir -p gpurun_out
export TMPDIR=/tmp
i=0
for C in "TCC_HIT_sum TCC_MISS_sum" "FETCH_SIZE" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY" "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d gpurun_out/${TAG}_$i -o run -- python tools/bench_wide.py pmc --only "$SH" > gpurun_out/${TAG}_$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 gpurun_out/${TAG}_$i.log; exit 1; }
  python tools/pmc_kernel.py gpurun_out/${TAG}_$i gemm_wide_kernel
done
