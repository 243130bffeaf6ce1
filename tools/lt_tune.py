"""Time the hipBLASLt heuristic's candidates for every library GEMM of the bench's BERT train step (B = 64 x L = 128
rows, bf16) with vcg_lt_tune, and print per shape the candidate that ran fastest and whether it beats candidate 0 (the
one the product path runs) by more than --margin. usage: python tools/lt_tune.py [--reps R] [--margin 0.05]"""
import argparse
import ctypes
import json
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "video-chapter-generation_amd"))
from vcg_hip import _lib  # noqa: E402
from vcg_hip.ops import P, stream  # noqa: E402

R, H, I = 8192, 768, 3072
# (name, transA, transB, M, N, K, lda, ldb, ldc, ldd, d_f32, bias, beta): the keys bert.py's calls produce
SHAPES = [
    ("qkv fwd", 0, 0, R, 3 * H, H, H, H, 0, 3 * H, 0, 1, 0.0),
    ("out-proj fwd", 0, 0, R, H, H, H, H, 0, H, 0, 1, 0.0),
    ("ffn1 fwd (pre)", 0, 0, R, I, H, H, H, 0, I, 0, 1, 0.0),
    ("ffn2 fwd", 0, 0, R, H, I, I, I, 0, H, 0, 1, 0.0),
    ("ffn1 dX +res", 0, 0, R, H, I, I, I, H, H, 0, 0, 1.0),
    ("out-proj dX", 0, 0, R, H, H, H, H, 0, H, 0, 0, 0.0),
    ("qkv dX +res", 0, 0, R, H, 3 * H, 3 * H, 3 * H, H, H, 0, 0, 1.0),
    ("ffn2 dW", 1, 1, H, I, R, H, I, I, I, 1, 0, 1.0),
    ("ffn1 dW", 1, 1, I, H, R, I, H, H, H, 1, 0, 1.0),
    ("out-proj dW", 1, 1, H, H, R, H, H, H, H, 1, 0, 1.0),
    ("qkv dW", 1, 1, 3 * H, H, R, 3 * H, H, H, H, 1, 0, 1.0),
]


def key(s):
    _, tA, tB, M, N, K, lda, ldb, ldc, ldd, f32, bias, beta = s
    return f"{tA},{tB},{M},{N},{K},{lda},{ldb},{ldc if beta else 0},{ldd},{f32},{bias},{1 if beta else 0}"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--margin", type=float, default=0.05)
    a = ap.parse_args()
    _lib.call("vcg_init", 0)
    dev = "cuda"
    table = {}
    for s in SHAPES:
        name, tA, tB, M, N, K, lda, ldb, ldc, ldd, f32, bias, beta = s
        A = torch.randn((K if tA else M) * lda, device=dev).to(torch.bfloat16)
        B = torch.randn((K if tB else N) * ldb, device=dev).to(torch.bfloat16) * 0.02
        D = torch.zeros(M * ldd, device=dev, dtype=torch.float32 if f32 else torch.bfloat16)
        C = torch.zeros(M * max(ldc, 1), device=dev, dtype=D.dtype) if beta else None
        bv = torch.zeros(N, device=dev) if bias else None
        us = (ctypes.c_float * 16)()
        n = _lib.lib().vcg_lt_tune(tA, tB, M, N, K, P(A), lda, P(B), ldb, P(C), ldc, P(D), ldd, f32, P(bv),
                                   ctypes.c_float(beta), a.reps, ctypes.addressof(us), 16, stream())
        t = [us[i] for i in range(max(n, 0))]
        fl = 2.0 * M * N * K
        ok = [(v, i) for i, v in enumerate(t) if v > 0]
        best = min(ok) if ok else (None, 0)
        pick = best[1] if ok and best[0] < t[0] * (1 - a.margin) else 0
        print(f"{name:16s} n={n:2d} cand0 {t[0] if t else -1:7.1f}us ({fl / max(t[0], 1e-9) / 1e6 if t else 0:5.0f} TF/s)"
              f"  best #{best[1]} {best[0] if best[0] else -1:7.1f}us  -> pick {pick}   all: "
              + " ".join(f"{v:.1f}" for v in t), flush=True)
        if pick:
            table[key(s)] = {"pick": pick, "name": name, "us_cand0": round(t[0], 1), "us_pick": round(t[pick], 1)}
    print(json.dumps(table, indent=1))


if __name__ == "__main__":
    main()
