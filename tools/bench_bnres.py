"""Time the bn3 GEMM pass (vcg_conv1x1_bn_res_relu: relu(bf16(a2 wfold^T + bias) + res) + mask bits) at the trunk's
shapes on the register-streaming kernel (VCG_RS1X1=1) and the persistent engine (0), same process.
usage: python tools/bench_bnres.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "video-chapter-generation_amd"))
from vcg_hip import _lib, ops  # noqa: E402

_lib.call("vcg_init", 0)
dev, bf = "cuda", torch.bfloat16
for name, M, K, N in (("l1", 3211264, 64, 256), ("l2", 802816, 128, 512), ("l3", 200704, 256, 1024)):
    x = torch.randn(M, K, device=dev).relu().to(bf)
    wf = (torch.randn(N, K, device=dev) / K ** 0.5).to(bf)
    b = torch.randn(N, device=dev) * 0.1
    res = torch.randn(M, N, device=dev).to(bf)
    gb = (M * K * 2 + 2 * M * N * 2 + M * N / 8) / 1e9
    for flag in ("1", "0", "1", "0"):
        os.environ["VCG_RS1X1"] = flag
        for _ in range(3):
            ops.conv1x1_bn_res_relu(x, wf, b, res, M, N, K)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            ops.conv1x1_bn_res_relu(x, wf, b, res, M, N, K)
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / 10 * 1e3
        print(f"{name} M={M} K={K} N={N} VCG_RS1X1={flag}: {us:8.1f} us  {gb / us * 1e3:5.2f} TB/s", flush=True)
