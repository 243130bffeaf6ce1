"""Time the small per-block kernels of the trunk backward / forward at the bench shapes (HIP events, 20 launches):
the bn3 fold weights (vcg_bn_bwd_fold_weights_a2), its weight-gradient combine (vcg_bn_bwd_fold_wgrad_a2) and the
Gram statistics (vcg_bn_stats_from_gram). usage: python tools/bench_small.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "video-chapter-generation_amd"))
from vcg_hip import _lib, ops  # noqa: E402

_lib.call("vcg_init", 0)
dev = "cuda"


def timeit(fn, n=20):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(n):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / n * 1e3


for C, K, M in ((64, 256, 3211264), (128, 512, 802816), (256, 1024, 200704)):
    g = torch.Generator(device=dev).manual_seed(C)
    wt = (torch.randn(C, K, device=dev, generator=g) / K ** 0.5).to(torch.bfloat16)
    v = lambda n, s=1.0: torch.rand(n, device=dev, generator=g) * s + 0.5  # noqa: E731
    invstd, gamma, sg, sgx, cs = v(K), v(K), v(K), v(K), v(C, 100.0)
    t1 = timeit(lambda: ops.bn_bwd_fold_weights_a2(wt, C, K, invstd, gamma, sg, sgx, M, cs))
    Pg, G, w3 = (torch.randn(K, C, device=dev, generator=g), torch.randn(C, C, device=dev, generator=g),
                 torch.randn(K, C, device=dev, generator=g))
    dw = torch.zeros(K, C, device=dev)
    t2 = timeit(lambda: ops.bn_bwd_fold_wgrad_a2(Pg, G, w3, K, C, v(K), invstd, gamma, sg, sgx, M, cs, dw))
    print(f"C={C} K={K}: fold_weights_a2 {t1:7.1f} us   fold_wgrad_a2 {t2:7.1f} us (incl. one small rand)", flush=True)
