"""Time the stem's streaming passes at the bench shape (1024 frames, 112x112x64 bf16 conv output): the fused
bn_relu_maxpool / maxpool_bwd_bn(sums only) + maxpool_bwd_bn_apply vs bn_apply + maxpool_fwd / maxpool_bwd_bn +
bn_bwd_apply. usage: python tools/bench_stem.py [N]"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "video-chapter-generation_amd"))
from vcg_hip import _lib, ops  # noqa: E402

_lib.call("vcg_init", 0)
N = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
H = W = 112
C = 64
dev = "cuda"
bf = torch.bfloat16
y = torch.randn(N, H, W, C, device=dev).to(bf)
sc = torch.rand(C, device=dev) + 0.5
sh = torch.randn(C, device=dev) * 0.2
mean = torch.zeros(C, device=dev)
inv = torch.ones(C, device=dev)
gamma = torch.ones(C, device=dev)
mp, idx = ops.bn_relu_maxpool(y, sc, sh, N, H, W, C)
dmp = torch.randn_like(mp)
sums = torch.zeros((2, C), device=dev)


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


res = {
    "fwd fused bn_relu_maxpool": t(lambda: ops.bn_relu_maxpool(y, sc, sh, N, H, W, C)),
    "fwd unfused bn_apply": t(lambda: ops.bn_apply(y, sc, sh, C, relu=True)),
    "fwd unfused maxpool_fwd": t(lambda: ops.maxpool_fwd(y, N, H, W, C)),
    "bwd sums-only maxpool_bwd_bn": t(lambda: ops.maxpool_bwd_bn(dmp, idx, N, H, W, C, y, mean, inv, sc, sh, sums,
                                                                 store_g=False)),
    "bwd apply maxpool_bwd_bn_apply": t(lambda: ops.maxpool_bwd_bn_apply(dmp, idx, N, H, W, C, y, mean, inv, sc, sh,
                                                                         gamma, sums, N * H * W, True)),
    "bwd unfused maxpool_bwd_bn (g stored)": t(lambda: ops.maxpool_bwd_bn(dmp, idx, N, H, W, C, y, mean, inv, sc, sh,
                                                                          sums)),
    "bwd unfused bn_bwd_apply": t(lambda: ops.bn_bwd_apply(y, None, y, mean, inv, gamma, sums[0], sums[1], C, True)),
}
for k, v in res.items():
    print(f"{k:40s} {v:8.1f} us", flush=True)
