"""Micro-benchmark of the fused conv-dgrad epilogue (vcg_conv_dgrad_bwd, EPI_BWD) on the train step's
heaviest shapes (profiles/r01_gemm_breakdown.txt), HIP events, bf16. Prints us per launch and the
effective HBM rate of the algorithmic bytes (dy + g + res + y (+ y2) + mask bits).
usage: python tools/bench_dgrad_bwd.py"""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "video-chapter-generation_amd"))
from vcg_hip import _lib, ops  # noqa: E402

DEV = "cuda"
# (name, frames, H, C (dgrad output = conv input channels), Cout, k, stride, pad, mode)
CASES = [
    ("l1.conv1 256<-64 tsm+bits", 1024, 56, 256, 64, 1, 1, 0, "tsm_bits"),
    ("l1.conv1 256<-64 bits (no TSM)", 1024, 56, 256, 64, 1, 1, 0, "bits"),
    ("l1.b1 conv1 tsm+bits+y2", 1024, 56, 256, 64, 1, 1, 0, "tsm_bits_two"),
    ("l2.conv1 512<-128 tsm+bits", 1024, 28, 512, 128, 1, 1, 0, "tsm_bits"),
    ("l2.conv1 512<-128 bits (no TSM)", 1024, 28, 512, 128, 1, 1, 0, "bits"),
    ("l1.conv2 3x3 64<-64 affine", 1024, 56, 64, 64, 3, 1, 1, "affine"),
    ("l1.conv3 64<-256 affine", 1024, 56, 64, 256, 1, 1, 0, "affine"),
    ("l3.conv1 1024<-256 tsm+bits", 1024, 14, 1024, 256, 1, 1, 0, "tsm_bits"),
    ("l2.b0 conv1 256<-128 tsm", 1024, 56, 256, 128, 1, 1, 0, "tsm_bits_two"),
]


def timeit(fn, iters=10):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


def main():
    _lib.call("vcg_init", 0)
    dt = torch.bfloat16
    tot = 0.0
    for name, N, H, C, Cout, k, s, p, mode in CASES:
        W = H
        OH, OW = ops.conv_out_hw(H, W, k, k, s, p)
        dy = torch.randn((N, OH, OW, Cout), device=DEV).to(dt)
        wt = ops.weight_prep(torch.randn((Cout, C, k, k), device=DEV) * 0.05, C, dt, transposed=True)
        y = torch.randn((N, H, W, C), device=DEV).to(dt)
        mean, inv = torch.zeros(C, device=DEV), torch.ones(C, device=DEV)
        sums = torch.zeros((2, C), device=DEV)
        dg, db = torch.zeros(C, device=DEV), torch.zeros(C, device=DEV)
        el = N * H * W * C
        if mode == "affine":
            msc, msh = torch.ones(C, device=DEV), torch.zeros(C, device=DEV)

            def fn():
                ops.conv_dgrad_bwd(dy, wt, N, H, W, C, Cout, k, k, s, p, y=y, mean=mean, invstd=inv, mscale=msc,
                                   mshift=msh, sums=sums, dgamma=dg, dbeta=db)
            nbytes = dy.numel() * 2 + el * 2 * 2
        else:
            res = torch.randn((N, H, W, C), device=DEV).to(dt)
            _, bits = ops.bn_apply(y, torch.ones(C, device=DEV), torch.zeros(C, device=DEV), C, relu=True, bits=True)
            tsm = mode.startswith("tsm")
            kw = dict(tsm_T=16 if tsm else 0, tsm_fold=C // 8 if tsm else 0, res=res, bits=bits, y=y, mean=mean,
                      invstd=inv, sums=sums, dgamma=dg, dbeta=db)
            nbytes = dy.numel() * 2 + el * 2 * 3 + el // 8
            if mode == "tsm_bits_two":
                y2 = torch.randn((N, H, W, C), device=DEV).to(dt)
                sgx2, dg2, db2 = (torch.zeros(C, device=DEV) for _ in range(3))
                kw.update(y2=y2, mean2=mean, invstd2=inv, sum_gx2=sgx2, dgamma2=dg2, dbeta2=db2)
                nbytes += el * 2

            def fn():
                ops.conv_dgrad_bwd(dy, wt, N, H, W, C, Cout, k, k, s, p, **kw)
        us = timeit(fn)
        tot += us
        fl = 2.0 * N * H * W * C * Cout * k * k
        print(f"{name:32s} {us:8.1f} us  {nbytes / us / 1e3:7.1f} GB/s  {fl / us / 1e6:7.1f} TF/s", flush=True)
    print(f"total {tot:.1f} us")


if __name__ == "__main__":
    main()
