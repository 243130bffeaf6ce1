"""Run one conv shape through the fast GEMM N times (for rocprofv3 --pmc stall breakdowns).
usage: one_gemm.py [shape] where shape in l3c2 (3x3 256->256 @14x14) | l1c3 (1x1 64->256 @56x56, stats)"""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "video-chapter-generation_amd"))
from vcg_hip import ops, _lib  # noqa: E402

SHAPES = {"l3c2": (1024, 14, 14, 256, 256, 3, 1, 1, True), "l1c3": (1024, 56, 56, 64, 256, 1, 1, 0, True),
          "l2c2": (1024, 28, 28, 128, 128, 3, 1, 1, True)}


def main():
    _lib.call("vcg_init", 0)
    name = sys.argv[1] if len(sys.argv) > 1 else "l3c2"
    N, H, W, C, Co, k, s, p, st = SHAPES[name]
    dt = torch.bfloat16
    x = torch.randn(N, H, W, C, device="cuda").to(dt)
    w = (torch.randn(Co, k, k, C, device="cuda") * 0.05).to(dt)
    OH, OW = ops.conv_out_hw(H, W, k, k, s, p)
    stats = ops.stats_buffer(Co, N * OH * OW, "cuda") if st else None
    y = torch.empty((N, OH, OW, Co), dtype=dt, device="cuda")
    for _ in range(10):
        ops.conv_fwd(x, w, N, H, W, C, Co, k, k, s, p, 0, 0, stats=stats, out=y)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
