"""Time the trunk's fused 1x1 conv1 input gradients (EPI_BWD: TSM adjoint + residual + mask bits + BN3 sums,
igemm_fast_kernel) at the bench shapes; with a -DVCG_FAST_STAMPS build (VCG_LIB_PATH=...) also print the per-tile
phase stamps of workgroup 0. usage: python tools/bench_dgrad.py"""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "video-chapter-generation_amd"))
from vcg_hip import _lib, ops  # noqa: E402

_lib.call("vcg_init", 0)
NOTSM = os.environ.get("VCG_BENCH_NOTSM") == "1"
NOY = os.environ.get("VCG_BENCH_NOY") == "1"  # mask bits without y (the trunk's y3-drop blocks: XF_BITS)
dev, bf = "cuda", torch.bfloat16
SHAPES = [  # (name, N, H, W, C (dx channels), Cout (dy channels), T, residual stride)
    ("l1 conv1 dgrad", 1024, 56, 56, 256, 64, 16, 1),
    ("l2 b0 conv1 dgrad", 1024, 56, 56, 256, 128, 16, 2),
    ("l2 conv1 dgrad", 1024, 28, 28, 512, 128, 16, 1),
    ("l3 conv1 dgrad", 1024, 14, 14, 1024, 256, 16, 1),
    ("l3 b0 conv1 dgrad", 1024, 28, 28, 512, 256, 16, 2),
]


def run(name, N, H, W, C, Co, T, rs=1):
    dy = torch.randn(N, H, W, Co, device=dev).to(bf)
    wt = ops.weight_prep((torch.randn(Co, C, 1, 1, device=dev) * 0.05), C, bf, transposed=True)
    res = torch.randn(N, (H + 1) // rs, (W + 1) // rs, C, device=dev).to(bf) if rs == 2 else \
        torch.randn(N, H, W, C, device=dev).to(bf)
    y = torch.randn(N, H, W, C, device=dev).to(bf)
    _, bits = ops.bn_apply(y, torch.ones(C, device=dev), torch.zeros(C, device=dev), C, relu=True, bits=True)
    mean, inv = torch.zeros(C, device=dev), torch.ones(C, device=dev)
    sums = torch.zeros((2, C), device=dev)
    dg, db = torch.zeros(C, device=dev), torch.zeros(C, device=dev)
    out = torch.empty(N, H, W, C, device=dev, dtype=bf)
    wsb = ops.ws(_lib.query("vcg_conv_dgrad_bwd_ws_bytes", C, Co, 1, 1), dev)

    def f():
        ops.conv_dgrad_bwd(dy, wt, N, H, W, C, Co, 1, 1, 1, 0, tsm_T=T, tsm_fold=0 if NOTSM else C // 8, res=res, res_stride=rs, bits=bits, y=None if NOY else y,
                           mean=mean, invstd=inv, sums=sums, dgamma=dg, dbeta=db, out=out, workspace=wsb)
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(10):
        f()
    b.record()
    torch.cuda.synchronize()
    us = a.elapsed_time(b) / 10 * 1e3
    M = N * H * W
    gb = (M * Co + (1 + (0 if NOY else 1) + (0.25 if rs == 2 else 1)) * M * C) * 2 / 1e9 + M * C / 8 / 1e9  # dy + y + g + res + bits
    line = f"{name:16s} M={M} N={C} K={Co}: {us:8.1f} us  {gb / us * 1e3:6.2f} TB/s algorithmic"
    buf = (ctypes.c_ulonglong * 256)()
    if _lib.query("vcg_fast_stamps", ctypes.addressof(buf), 256) == 0:
        f()
        torch.cuda.synchronize()
        _lib.query("vcg_fast_stamps", ctypes.addressof(buf), 256)
        st = np.frombuffer(buf, dtype=np.uint64).astype(np.int64).reshape(64, 4)
        n = int((st[:, 0] > 0).sum())
        st = st[2:max(3, n - 2)]
        per = np.diff(st[:, 0])
        d = np.diff(st, axis=1)
        line += (f" | stamps over {len(per)} tiles: per-tile {per.mean():.0f} ticks; mfma {d[:, 0].mean():.0f} stage "
                 f"{d[:, 1].mean():.0f} flush {d[:, 2].mean():.0f} next-tile wait {(per - (st[:-1, 3] - st[:-1, 0])).mean():.0f}")
    print(line, flush=True)


# argv: [name prefix] [comma-separated VCG_BWD_STREAM values: 1 (streaming), 64 (streaming, 64-column tiles), 0]; VCG_BENCH_NOTSM=1: no TSM adjoint (A/B of the access pattern)
sel = sys.argv[1] if len(sys.argv) > 1 else ""
flags = sys.argv[2].split(",") if len(sys.argv) > 2 else ["1", "0"]  # VCG_BWD_STREAM values, e.g. 1,64,0
for s in SHAPES:  # the streaming kernel (EPI_BWD_STREAM, K <= 128) and the persistent engine, same process
    if not s[0].startswith(sel):
        continue
    for flag in flags:
        os.environ["VCG_BWD_STREAM"] = flag
        print(f"VCG_BWD_STREAM={flag} ", end="")
        run(*s)
