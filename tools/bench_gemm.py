"""Micro-benchmark of single libvcg_hip GEMM / conv shapes (HIP events, bf16), with a device copy
as the bandwidth reference. Usage: python tools/bench_gemm.py"""
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
    if os.environ.get("VCG_BENCH_STAMPS"):  # per-tile phase stamps of workgroup 0 (a -DVCG_FAST_STAMPS build)
        import ctypes
        import numpy as np
        from vcg_hip import _lib
        for name, fn in _ab_cases() + _dense_cases():
            us = timeit(fn, 5)
            buf = (ctypes.c_ulonglong * 256)()
            if _lib.query("vcg_fast_stamps", ctypes.addressof(buf), 256) != 0:
                print("not a stamps build")
                return
            st = np.frombuffer(buf, dtype=np.uint64).astype(np.int64).reshape(64, 4)
            n = int((st[:, 0] > 0).sum())
            st = st[1:max(2, n - 1)]
            per = np.diff(st[:, 0])
            d = np.diff(st, axis=1)
            print(f"{name:32s} {us:7.1f} us | {len(per)} tiles: per-tile {per.mean():6.0f} ticks: k-loop {d[:, 0].mean():6.0f} "
                  f"stage {d[:, 1].mean():5.0f} flush {d[:, 2].mean():5.0f} to next tile {(per - (st[:-1, 3] - st[:-1, 0])).mean():5.0f}",
                  flush=True)
        return
    if os.environ.get("VCG_BENCH_AB"):  # A/B of the output staging threshold in one process
        for name, fn in _ab_cases():
            res = []
            for kt in ("0", "4", "1000"):
                os.environ["VCG_STAGE_KT"] = kt
                res.append(f"stage_kt={kt}: {timeit(fn, 20):8.1f}us")
            print(f"{name:32s} " + "  ".join(res))
        return

    dt = torch.bfloat16
    dev = "cuda"
    a = torch.empty(800 * 1024 * 1024, dtype=torch.uint8, device=dev)
    b = torch.empty_like(a)
    us = timeit(lambda: b.copy_(a))
    print(f"copy 800MiB: {us:8.1f} us  {2 * a.numel() / us / 1e3:7.1f} GB/s (read+write)")
    rows = []
    # (name, N, H, W, C, Cout, k, stride, pad, tsm, stats)
    convs = [
        ("l1 conv3 1x1 64->256", 1024, 56, 56, 64, 256, 1, 1, 0, 0, True),
        ("l1 conv3 1x1 64->256 nostats", 1024, 56, 56, 64, 256, 1, 1, 0, 0, False),
        ("l1 conv1 1x1 256->64 tsm", 1024, 56, 56, 256, 64, 1, 1, 0, 16, True),
        ("l1 conv2 3x3 64->64", 1024, 56, 56, 64, 64, 3, 1, 1, 0, True),
        ("l2 conv2 3x3 128->128", 1024, 28, 28, 128, 128, 3, 1, 1, 0, True),
        ("l3 conv1 1x1 1024->256", 1024, 14, 14, 1024, 256, 1, 1, 0, 0, True),
        ("l3 conv2 3x3 256->256", 1024, 14, 14, 256, 256, 3, 1, 1, 0, True),
        ("l4 conv3 1x1 512->2048", 1024, 7, 7, 512, 2048, 1, 1, 0, 0, True),
        ("stem 7x7/2 8->64", 1024, 224, 224, 8, 64, 7, 2, 3, 0, True),
    ]
    for name, N, H, W, C, Co, k, s, p, tsm, st in convs:
        x = torch.randn(N, H, W, C, device=dev).to(dt)
        w = torch.randn(Co, k, k, C, device=dev).to(dt) * 0.05
        OH, OW = ops.conv_out_hw(H, W, k, k, s, p)
        M = N * OH * OW
        stats = ops.stats_buffer(Co, M, dev) if st else None
        y = torch.empty((N, OH, OW, Co), dtype=dt, device=dev)
        fold = C // 8 if tsm else 0
        us = timeit(lambda: ops.conv_fwd(x, w, N, H, W, C, Co, k, k, s, p, tsm, fold, stats=stats, out=y))
        fl = 2.0 * M * Co * k * k * C
        by = (x.numel() + y.numel()) * 2
        print(f"{name:32s} {us:8.1f} us  {fl / us / 1e6:7.1f} TF/s  {by / us / 1e3:7.1f} GB/s")
        del x, y
    # dgrad of the 1x1 conv1 of layer1 (dy 64 -> dx 256): K = 64, N = 256
    dy = torch.randn(1024, 56, 56, 64, device=dev).to(dt)
    wt = torch.randn(256, 1, 1, 64, device=dev).to(dt)
    dx = torch.empty(1024, 56, 56, 256, device=dev, dtype=dt)
    us = timeit(lambda: ops.conv_dgrad(dy, wt, 1024, 56, 56, 256, 64, 1, 1, 1, 0, out=dx))
    print(f"{'l1 dgrad 1x1 64->256':32s} {us:8.1f} us  {2.0 * dx.numel() * 64 / us / 1e6:7.1f} TF/s  "
          f"{(dy.numel() + dx.numel()) * 2 / us / 1e3:7.1f} GB/s")
    # BERT attention (B=64, 12 heads, L=128, dh=64) as the encoder calls it
    Bb, nh, L, dh = 64, 12, 128, 64
    H = nh * dh
    qkv = torch.randn(Bb * L, 3 * H, device=dev).to(dt)
    S = torch.empty((Bb * nh, L, L), dtype=dt, device=dev)
    us = timeit(lambda: ops.gemm_batched(qkv, qkv[:, H:], S, L, L, dh, 3 * H, 3 * H, L, L * 3 * H, dh, L * 3 * H, dh,
                                         nh * L * L, L * L, Bb, nh))
    print(f"{'attn QK^T batched':32s} {us:8.1f} us  {2.0 * Bb * nh * L * L * dh / us / 1e6:7.1f} TF/s")
    ctx = torch.empty((Bb * L, H), dtype=dt, device=dev)
    us = timeit(lambda: ops.gemm_batched(S, qkv[:, 2 * H:], ctx, L, dh, L, L, 3 * H, H, nh * L * L, L * L, L * 3 * H,
                                         dh, L * H, dh, Bb, nh, transB=True))
    print(f"{'attn PV batched (transB)':32s} {us:8.1f} us  {2.0 * Bb * nh * L * L * dh / us / 1e6:7.1f} TF/s")
    # BERT FFN1 / FFN2 / QKV
    for M, Nn, K in ((8192, 3072, 768), (8192, 768, 3072), (8192, 2304, 768), (8192, 8192, 8192),
                     (65536, 256, 2304), (65536, 128, 1152)):
        A = torch.randn(M, K, device=dev).to(dt)
        B = torch.randn(Nn, K, device=dev).to(dt)
        C = torch.empty(M, Nn, device=dev, dtype=dt)
        us = timeit(lambda: ops.gemm(A, B, M, Nn, K, K, K, out=C))
        print(f"gemm {M}x{Nn}x{K:<20d} {us:8.1f} us  {2.0 * M * Nn * K / us / 1e6:7.1f} TF/s")


def _dense_cases():
    dt, dev = torch.bfloat16, "cuda"
    out = []
    for M, Nn, K in ((8192, 3072, 768), (8192, 768, 3072), (200704, 1024, 256), (50176, 2048, 512)):
        A = torch.randn(M, K, device=dev).to(dt)
        B = torch.randn(Nn, K, device=dev).to(dt)
        C = torch.empty(M, Nn, device=dev, dtype=dt)
        out.append((f"gemm {M}x{Nn}x{K}", (lambda A=A, B=B, C=C, M=M, Nn=Nn, K=K: ops.gemm(A, B, M, Nn, K, K, K, out=C))))
    return out


def _ab_cases():
    dt = torch.bfloat16
    dev = "cuda"
    out = []
    for name, N, H, W, C, Co, k, s, p, st in (("l1 conv3 64->256 stats", 1024, 56, 56, 64, 256, 1, 1, 0, True),
                                              ("l1 conv3 64->256", 1024, 56, 56, 64, 256, 1, 1, 0, False),
                                              ("l2 conv3 128->512 stats", 1024, 28, 28, 128, 512, 1, 1, 0, True),
                                              ("l3 conv1 1024->256 stats", 1024, 14, 14, 1024, 256, 1, 1, 0, True),
                                              ("l2 conv2 3x3 128 stats", 1024, 28, 28, 128, 128, 3, 1, 1, True),
                                              ("l3 conv2 3x3 256 stats", 1024, 14, 14, 256, 256, 3, 1, 1, True),
                                              ("l3 conv3 256->1024 stats", 1024, 14, 14, 256, 1024, 1, 1, 0, True),
                                              ("l4 conv2 3x3 512 stats", 1024, 7, 7, 512, 512, 3, 1, 1, True)):
        x = torch.randn(N, H, W, C, device=dev).to(dt)
        w = torch.randn(Co, k, k, C, device=dev).to(dt) * 0.05
        OH, OW = ops.conv_out_hw(H, W, k, k, s, p)
        stats = ops.stats_buffer(Co, N * OH * OW, dev) if st else None
        y = torch.empty((N, OH, OW, Co), dtype=dt, device=dev)
        out.append((name, (lambda x=x, w=w, y=y, stats=stats, N=N, H=H, W=W, C=C, Co=Co, k=k, s=s, p=p:
                           ops.conv_fwd(x, w, N, H, W, C, Co, k, k, s, p, 0, 0, stats=stats, out=y))))
    return out


if __name__ == "__main__":
    main()
