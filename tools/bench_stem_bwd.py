"""Time the stem backward after the max-pool at the bench shape (N = 1024 frames, 112 x 112 conv output, 64
channels): the one-pass vcg_stem_bwd_fused against vcg_maxpool_bwd_bn_apply + the pair-packed im2col weight
gradient. usage: python tools/bench_stem_bwd.py [N]"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "video-chapter-generation_amd"))
from vcg_hip import _lib, ops  # noqa: E402

_lib.call("vcg_init", 0)
N = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
H1 = W1 = 112
C = 64
dev, bf = "cuda", torch.bfloat16
y = torch.randn(N, H1, W1, C, device=dev).to(bf)
sc = torch.rand(C, device=dev) + 0.5
sh = torch.randn(C, device=dev) * 0.1
mp, idx = ops.bn_relu_maxpool(y, sc, sh, N, H1, W1, C)
dys = torch.randn(mp.shape, device=dev).to(bf)
mean, inv, gamma = torch.zeros(C, device=dev), torch.ones(C, device=dev), torch.ones(C, device=dev)
sums = torch.zeros((2, C), device=dev)
ops.maxpool_bwd_bn(dys, idx, N, H1, W1, C, y, mean, inv, sc, sh, sums, store_g=False)
xs = torch.randn(N, 2 * H1, 2 * W1, 4, device=dev).to(bf)
dw = torch.zeros((C, 3, 7, 7), device=dev)
wsb = None


def unfused():
    global wsb
    dy0 = ops.maxpool_bwd_bn_apply(dys, idx, N, H1, W1, C, y, mean, inv, sc, sh, gamma, sums, N * H1 * W1, True)
    wsb = ops.conv_wgrad(xs, dy0, dw, N, 2 * H1, 2 * W1, 4, 3, C, 7, 7, 2, 3, workspace=wsb)


def fused():
    ops.stem_bwd_fused(dys, idx, y, xs, N, H1, W1, mean, inv, sc, sh, gamma, sums, N * H1 * W1, True, dw)


def t(fn, reps=10):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e3


gb = (y.numel() * 2 + dys.numel() * 2 + idx.numel() + xs.numel() * 2) / 1e9
for name, fn in (("apply + im2col wgrad", unfused), ("fused", fused)):
    us = t(fn)
    print(f"{name:22s} {us:8.1f} us   ({gb:.2f} GB read once: {gb / us * 1e3:.2f} TB/s)", flush=True)
