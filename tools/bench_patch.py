"""Time the layer-1 3x3 conv (M = 1024 x 56 x 56, C = 64 -> 64) fwd+stats and fused dgrad (EPI_BWD_AFF) on the
im2col engine vs the LDS-patch kernel (VCG_PATCH_OCC 2 / 1). usage: python tools/bench_patch.py [N]"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "video-chapter-generation_amd"))
from vcg_hip import _lib, ops  # noqa: E402

_lib.call("vcg_init", 0)
N = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
H = W = 56
C = 64
dev = "cuda"
bf = torch.bfloat16
x = torch.randn(N, H, W, C, device=dev).to(bf)
w = (torch.randn(C, C, 3, 3, device=dev) * 0.05)
wd = ops.weight_prep(w, C, bf)
wt = ops.weight_prep(w, C, bf, transposed=True)
M = N * H * W
st = ops.stats_buffer(C, M, dev)
y = torch.randn(N, H, W, C, device=dev).to(bf)
mean = torch.zeros(C, device=dev)
inv = torch.ones(C, device=dev)
msc = torch.ones(C, device=dev)
msh = torch.zeros(C, device=dev)
sums = torch.zeros((2, C), device=dev)
dg, db = torch.zeros(C, device=dev), torch.zeros(C, device=dev)
out = torch.empty_like(x)
wsb = ops.ws(_lib.query("vcg_conv_dgrad_bwd_ws_bytes", C, C, 3, 3), dev)


def fwd():
    ops.conv_fwd(x, wd, N, H, W, C, C, 3, 3, 1, 1, stats=st, out=out)


def dgrad():
    ops.conv_dgrad_bwd(x, wt, N, H, W, C, C, 3, 3, 1, 1, y=y, mean=mean, invstd=inv, mscale=msc, mshift=msh,
                       sums=sums, dgamma=dg, dbeta=db, out=out, workspace=wsb)


def t(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e3


for name, env in [("im2col", {"VCG_NO_PATCH": "1"}), ("patch", {})]:
    for k in ("VCG_NO_PATCH", "VCG_PATCH_OCC"):
        os.environ.pop(k, None)
    os.environ.update(env)
    print(f"{name:12s} fwd+stats {t(fwd):7.1f} us   fused dgrad {t(dgrad):7.1f} us", flush=True)

# phase stamps of workgroup 0 / wave 0 (s_memtime): per tile top -> waited -> DMA issued -> MFMAs -> barrier -> epilogue
import ctypes  # noqa: E402
import numpy as np  # noqa: E402

os.environ.pop("VCG_NO_PATCH", None)
os.environ["VCG_PATCH_STAMPS"] = "1"

for name, fn in (("fwd+stats", fwd), ("fused dgrad", dgrad)):
    fn()
    torch.cuda.synchronize()
    buf = (ctypes.c_ulonglong * (64 * 6))()
    rc = _lib.query("vcg_patch_stamps", ctypes.addressof(buf), 64 * 6)
    st = np.frombuffer(buf, dtype=np.uint64).astype(np.int64).reshape(64, 6)
    d = np.diff(st, axis=1)[2:60]             # steady-state tiles
    tile = np.diff(st[:, 0])[2:60]
    print(f"{name}: rc {rc}  per-tile {tile.mean():.0f} ticks; phases wait {d[:, 0].mean():.0f}  dma-issue "
          f"{d[:, 1].mean():.0f}  mfma {d[:, 2].mean():.0f}  barrier {d[:, 3].mean():.0f}  epilogue {d[:, 4].mean():.0f}",
          flush=True)
