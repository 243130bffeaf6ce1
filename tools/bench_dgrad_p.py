"""Time the streaming conv1 dgrad with and without the g^T a2 product (vcg_conv_dgrad_bwd with a2) against the
weight-gradient GEMM it replaces, at the trunk shapes (mask bits, no y). usage: python tools/bench_dgrad_p.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "video-chapter-generation_amd"))
from vcg_hip import _lib, ops  # noqa: E402

_lib.call("vcg_init", 0)
dev, bf = "cuda", torch.bfloat16
SHAPES = [  # (name, N, H, W, C, Cout, T, res_stride, a2 columns)
    ("l1 b2 conv1 dgrad", 1024, 56, 56, 256, 64, 16, 1, 64),
    ("l2 b0 conv1 dgrad", 1024, 56, 56, 256, 128, 16, 2, 64),
    ("l2 conv1 dgrad", 1024, 28, 28, 512, 128, 16, 1, 128),
    ("l3 b0 conv1 dgrad", 1024, 28, 28, 512, 256, 16, 2, 128),
]


def timeit(fn, n=10):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(n):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / n * 1e3


for name, N, H, W, C, Co, T, rs, PJ in SHAPES:
    dy = torch.randn(N, H, W, Co, device=dev).to(bf)
    wt = ops.weight_prep(torch.randn(Co, C, 1, 1, device=dev) * 0.05, C, bf, transposed=True)
    res = (torch.randn(N, (H + 1) // 2, (W + 1) // 2, C, device=dev) if rs == 2 else
           torch.randn(N, H, W, C, device=dev)).to(bf)
    _, bits = ops.bn_apply(torch.randn(N, H, W, C, device=dev).to(bf), torch.ones(C, device=dev),
                           torch.zeros(C, device=dev), C, relu=True, bits=True)
    a2 = torch.relu(torch.randn(N, H, W, PJ, device=dev)).to(bf)
    mean, inv = torch.zeros(C, device=dev), torch.ones(C, device=dev)
    sums = torch.zeros((2, C), device=dev)
    out = torch.empty(N, H, W, C, device=dev, dtype=bf)
    pg = torch.empty(C, PJ, device=dev)
    pw = torch.empty(C, PJ, 1, 1, device=dev)
    kw = dict(tsm_T=T, tsm_fold=C // 8, res=res, res_stride=rs, bits=bits, mean=mean, invstd=inv, sums=sums, out=out)
    t0 = timeit(lambda: ops.conv_dgrad_bwd(dy, wt, N, H, W, C, Co, 1, 1, 1, 0, **kw))
    t1 = timeit(lambda: ops.conv_dgrad_bwd(dy, wt, N, H, W, C, Co, 1, 1, 1, 0, a2=a2, pg=pg, **kw))
    t2 = timeit(lambda: ops.conv_wgrad(a2, out, pw, N, H, W, PJ, PJ, C, 1, 1, 1, 0, accumulate=False))
    print(f"{name:18s}: dgrad {t0:7.1f} us, dgrad + P {t1:7.1f} us (+{t1 - t0:6.1f}), P GEMM {t2:7.1f} us", flush=True)
