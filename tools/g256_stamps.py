"""Phase timing of the 256-tile GEMM (igemm256.hip) from its s_memtime stamps: run with a -DVCG_G256_STAMPS build,
  make -C video-chapter-generation_amd/csrc EXTRA=-DVCG_G256_STAMPS OBJDIR=../build/obj_stamps \
       OUT=../vcg_hip/libvcg_hip_g256stamps.so
  VCG_LIB_PATH=.../libvcg_hip_g256stamps.so VCG_G256=1 python tools/g256_stamps.py
Per phase of k-tiles 8..15, waves 0 (group 0) and 4 (group 1, one barrier behind): R = fragment reads + LDS-DMA issue
(from the previous phase's end), B1 = first barrier wait, M = the MFMAs, B2 = second barrier wait (cycles)."""
import ctypes
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "video-chapter-generation_amd"))
from vcg_hip import _lib, ops  # noqa: E402


def report(name):
    buf = (ctypes.c_ulonglong * 256)()
    if _lib.query("vcg_g256_stamps", ctypes.addressof(buf), 256) != 0:
        print("not a stamps build")
        sys.exit(1)
    st = np.frombuffer(buf, dtype=np.uint64).astype(np.int64).reshape(2, 8, 4, 4)
    print(name)
    for w in range(2):
        flat = st[w].reshape(-1, 4)  # [phase][point]
        prev = np.concatenate([[flat[0, 0]], flat[:-1, 3]])
        R = flat[:, 0] - prev
        B1 = flat[:, 1] - flat[:, 0]
        M = flat[:, 2] - flat[:, 1]
        B2 = flat[:, 3] - flat[:, 2]
        per_tile = (flat[4::4, 3] - flat[0:-4:4, 3]).mean() if len(flat) > 4 else 0
        print(f"  wave {4 * w}: per k-tile {per_tile:7.0f} cyc | by phase q0..q3: R {R[4:].reshape(-1, 4).mean(0).round()} "
              f"B1 {B1.reshape(-1, 4).mean(0).round()} M {M.reshape(-1, 4).mean(0).round()} "
              f"B2 {B2.reshape(-1, 4).mean(0).round()}")


def main():
    _lib.call("vcg_init", 0)
    dev, dt = "cuda", torch.bfloat16
    M = N = K = 8192
    A = (torch.rand(M, K, device=dev) * 2 - 1).to(dt)
    B = ((torch.rand(N, K, device=dev) * 2 - 1) * 0.05).to(dt)
    C = torch.empty(M, N, dtype=dt, device=dev)
    for _ in range(3):
        ops.gemm(A, B, M, N, K, K, K, out=C)
    torch.cuda.synchronize()
    report("square 8192^3")
    x = (torch.rand(1024, 14, 14, 256, device=dev) * 2 - 1).to(dt)
    w = ((torch.rand(256, 3, 3, 256, device=dev) * 2 - 1) * 0.05).to(dt)
    y = torch.empty(1024, 14, 14, 256, dtype=dt, device=dev)
    for _ in range(3):
        ops.conv_fwd(x, w, 1024, 14, 14, 256, 256, 3, 3, 1, 1, out=y)
    torch.cuda.synchronize()
    report("l3 conv2 3x3 256")


if __name__ == "__main__":
    main()
