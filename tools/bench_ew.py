"""Micro-benchmark of the trunk's streaming kernels (BN apply, BN backward reduce / apply, TSM
gradient combine) at the B=64 x 16-frame shapes, bf16, HIP events; GB/s = algorithmic bytes
(each tensor read / written once) / time, next to a device copy. Usage: python tools/bench_ew.py"""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "video-chapter-generation_amd"))
from vcg_hip import ops  # noqa: E402


def timeit(fn, iters=10):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3  # us


def main():
    dt = torch.bfloat16
    dev = "cuda"
    a = torch.empty(1600 * 1024 * 1024, dtype=torch.uint8, device=dev)
    b = torch.empty_like(a)
    us = timeit(lambda: b.copy_(a))
    print(f"copy 1600MiB: {us:8.1f} us  {2 * a.numel() / us / 1e3:7.1f} GB/s (read+write)")
    del a, b
    NF = 1024
    for (HW, C) in ((3136, 256), (3136, 64), (784, 512), (196, 1024), (49, 2048)):
        P = NF * HW
        n = P * C
        y = (torch.randn(P, C, device=dev) * 0.5).to(dt)
        d = torch.randn(P, C, device=dev).to(dt)
        res = torch.randn(P, C, device=dev).to(dt)
        sc = torch.rand(C, device=dev) + 0.5
        sh = torch.randn(C, device=dev) * 0.1
        mean = torch.randn(C, device=dev) * 0.1
        inv = torch.rand(C, device=dev) + 0.5
        gamma = torch.rand(C, device=dev) + 0.5
        sums = torch.zeros(2, C, device=dev)
        out = torch.empty_like(y)
        nb = 2 * n
        line = [f"P={P:8d} C={C:5d} {nb / 2**20:7.0f} MiB/pass"]
        t = timeit(lambda: ops.bn_apply(y, sc, sh, C, relu=True, out=out))
        line.append(f"apply {t:7.1f}us {2 * nb / t / 1e3:6.0f}GB/s")
        t = timeit(lambda: ops.bn_apply(y, sc, sh, C, relu=True, res=res, out=out, bits=True))
        line.append(f"apply+res+bits {t:7.1f}us {(3 * nb + n // 8) / t / 1e3:6.0f}GB/s")
        wsb = ops.ws(ops._lib.query("vcg_bn_bwd_ws_bytes", P, C), dev)
        t = timeit(lambda: ops.bn_bwd_reduce(d, None, y, mean, inv, C, sums[0], sums[1], workspace=wsb,
                                             mscale=sc, mshift=sh))
        line.append(f"bwd_red {t:7.1f}us {2 * nb / t / 1e3:6.0f}GB/s")
        t = timeit(lambda: ops.bn_bwd_apply(d, None, y, mean, inv, gamma, sums[0], sums[1], C, train_stats=True,
                                            out=out, mscale=sc, mshift=sh))
        line.append(f"bwd_app {t:7.1f}us {3 * nb / t / 1e3:6.0f}GB/s")
        bits = torch.randint(0, 255, (n // 8,), dtype=torch.uint8, device=dev)
        t = timeit(lambda: ops.tsm_unshift_add(d, res, P // HW, 16, HW, C, C // 8, other_bits=bits))
        line.append(f"tsm {t:7.1f}us {(3 * nb + n // 8) / t / 1e3:6.0f}GB/s")
        print("  ".join(line), flush=True)
        del y, d, res, out


if __name__ == "__main__":
    main()
