"""Time the stride-1 3x3 weight gradients of the bench step (B=64 x T=16 frames) with HIP events: layer 1-4 shapes.
VCG_WGRAD_PATCH=1 keeps the patch kernel to layer 1 (the im2col engine elsewhere), =2 (default) uses it everywhere.
usage: VCG_WGRAD_PATCH=1|2 python tools/bench_wgrad3x3.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "video-chapter-generation_amd"))
from vcg_hip import _lib, ops  # noqa: E402

_lib.call("vcg_init", 0)
dev, bf = "cuda", torch.bfloat16
N = 1024
for (H, C) in ((56, 64), (28, 128), (14, 256), (7, 512)):
    x = torch.randn(N, H, H, C, device=dev).to(bf)
    dy = torch.randn(N, H, H, C, device=dev).to(bf)
    dw = torch.zeros((C, C, 3, 3), device=dev)
    wsb = ops.conv_wgrad(x, dy, dw, N, H, H, C, C, C, 3, 3, 1, 1)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(10):
        ops.conv_wgrad(x, dy, dw, N, H, H, C, C, C, 3, 3, 1, 1, workspace=wsb)
    b.record()
    torch.cuda.synchronize()
    us = a.elapsed_time(b) / 10 * 1e3
    fl = 2.0 * C * 9 * C * N * H * H
    print(f"VCG_WGRAD_PATCH={os.environ.get('VCG_WGRAD_PATCH', '2')} {H}x{H}x{C}: {us:7.1f} us  {fl / us / 1e6:6.0f} TF/s",
          flush=True)
    del x, dy
