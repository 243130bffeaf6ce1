"""Per-phase timing of the wide-tile GEMM engine from a -DVCG_WIDE_STAMPS build (tools/build_variant.sh): runs one
BERT GEMM shape with VCG_LIB_PATH pointing at the stamped library and prints, for waves 0 (group A) and 4 (group B)
of workgroup 0, the median cycles of each phase segment over k-steps 8..23:
  read phase:    reads+DMA issue | lgkmcnt wait | vmcnt wait | barrier (to the compute phase's top)
  compute phase: MFMAs | vmcnt wait | epilogue | barrier (to the next read phase's top)
usage: VCG_LIB_PATH=.../libvcg_wide_stamps.so python tools/wide_stamps.py [N K]"""
import ctypes
import os
import statistics
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "video-chapter-generation_amd"))
from vcg_hip import _lib, ops  # noqa: E402


def main():
    N, K = (int(sys.argv[1]), int(sys.argv[2])) if len(sys.argv) > 2 else (768, 3072)
    R = 8192
    A = torch.randn(R, K, device="cuda").to(torch.bfloat16)
    W = (torch.randn(N, K, device="cuda") * 0.02).to(torch.bfloat16)
    for _ in range(5):
        ops.gemm(A, W, R, N, K, K, K, act=ops.ACT_FLAG_WIDE)
    torch.cuda.synchronize()
    buf = (ctypes.c_ulonglong * 256)()
    rc = _lib.lib().vcg_wide_stamps(buf, 256)
    assert rc == 0, "not a stamped build"
    st = list(buf)
    for w, name in ((0, "wave 0 (A)"), (1, "wave 4 (B)")):
        rows = []
        for k in range(16):
            b = ((w * 16 + k) * 2) * 4
            r, c = st[b:b + 4], st[b + 4:b + 8]
            nxt = st[b + 8] if k < 15 else None
            rows.append((r[1] - r[0], r[2] - r[1], r[3] - r[2], c[0] - r[3], c[1] - c[0], c[2] - c[1], c[3] - c[2],
                         (nxt - c[3]) if nxt else 0, (nxt - r[0]) if nxt else 0))
        med = [statistics.median(x[i] for x in rows) for i in range(9)]
        print(f"{name}: read {med[0]:.0f} lgkm {med[1]:.0f} vm {med[2]:.0f} bar {med[3]:.0f} | "
              f"mfma {med[4]:.0f} vm {med[5]:.0f} epi {med[6]:.0f} bar {med[7]:.0f} | step {med[8]:.0f} cycles")


if __name__ == "__main__":
    main()
