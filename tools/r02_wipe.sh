#!/bin/bash
# is the slow bench after a big process the freed-VRAM clearing? A process that only allocates + touches 60 GB and
# exits, then the bench at once; then a 40 s pause and the bench again
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 120 python -c "
import torch, time
x = [torch.ones(2**30, dtype=torch.float32, device='cuda') for _ in range(15)]
torch.cuda.synchronize(); print('allocated', sum(t.numel() for t in x) * 4 / 2**30, 'GiB')
" || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/wipe_1.log 2>&1 || exit 1
echo "bench right after the 60 GB process: $(grep -o '"value": [0-9.]*' gpurun_out/wipe_1.log)"
sleep 40
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/wipe_2.log 2>&1 || exit 1
echo "bench 40 s after the previous bench: $(grep -o '"value": [0-9.]*' gpurun_out/wipe_2.log)"
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/wipe_3.log 2>&1 || exit 1
echo "bench right after the previous bench: $(grep -o '"value": [0-9.]*' gpurun_out/wipe_3.log)"
