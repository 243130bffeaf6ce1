"""Times the wide-tile engine on BERT-base's dense GEMMs at B=64 x L=128 (8192 rows), HIP events, 20 reps each, with
the library and environment it is started with (VCG_LIB_PATH, VCG_WIDE_BN): one line per shape plus
the sum over one BERT layer's forward + input gradients (x12 = per step).
usage: python tools/bench_wide.py [tag] [--only <shape name prefix>]"""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "video-chapter-generation_amd"))
from vcg_hip import ops  # noqa: E402


def timeit(fn, iters=20):
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
    only = sys.argv[sys.argv.index("--only") + 1] if "--only" in sys.argv else None
    args = [a for i, a in enumerate(sys.argv[1:], 1) if a != "--only" and sys.argv[i - 1] != "--only"]
    tag = args[0] if args else "default"
    dt, dev, W_ = torch.bfloat16, "cuda", ops.ACT_FLAG_WIDE
    R, H, I = 8192, 768, 3072
    g = torch.Generator(device=dev).manual_seed(0)

    def rnd(*s, sc=1.0):
        return (torch.randn(*s, device=dev, generator=g) * sc).to(dt)
    x, xi = rnd(R, H), rnd(R, I)
    shapes = []
    for (N, K, name) in ((3 * H, H, "qkv"), (H, H, "out"), (I, H, "ffn1"), (H, I, "ffn2")):
        W, b = rnd(N, K, sc=0.02), torch.zeros(N, device=dev)
        A = x if K == H else xi
        if name == "ffn1":
            pre = torch.empty(R, N, dtype=dt, device=dev)
            shapes.append((f"{name} fwd+gelu", 2.0 * R * N * K,
                           lambda A=A, W=W, b=b, N=N, K=K, pre=pre: ops.gemm(A, W, R, N, K, K, K, bias=b,
                                                                             act=ops.ACT_GELU | W_, aux=pre)))
        else:
            shapes.append((f"{name} fwd", 2.0 * R * N * K,
                           lambda A=A, W=W, b=b, N=N, K=K: ops.gemm(A, W, R, N, K, K, K, bias=b, act=W_)))
        dY, Wt = rnd(R, N), rnd(K, N, sc=0.02)  # dX [R, K] = dY [R, N] W [N, K]: W^T resident [K][N]
        if name == "ffn2":
            pre = rnd(R, K)
            shapes.append((f"{name} dX+gelu'", 2.0 * R * N * K,
                           lambda dY=dY, Wt=Wt, N=N, K=K, pre=pre: ops.gemm(dY, Wt, R, K, N, N, N,
                                                                            act=ops.ACT_GELU_BWD | W_, residual=pre,
                                                                            ldr=K)))
        else:
            r = rnd(R, K)
            shapes.append((f"{name} dX+res" if name != "out" else f"{name} dX", 2.0 * R * N * K,
                           (lambda dY=dY, Wt=Wt, N=N, K=K, r=r: ops.gemm(dY, Wt, R, K, N, N, N, residual=r, ldr=K,
                                                                        act=W_)) if name != "out" else
                           (lambda dY=dY, Wt=Wt, N=N, K=K: ops.gemm(dY, Wt, R, K, N, N, N, act=W_))))
    tot = 0.0
    parts = []
    for name, fl, fn in shapes:
        if only and not name.startswith(only):
            continue
        t = timeit(fn)
        tot += t
        parts.append(f"{name} {t:6.1f}us/{fl / t / 1e6:4.0f}")
    print(f"[{tag}] layer {tot:6.1f}us  " + "  ".join(parts), flush=True)


if __name__ == "__main__":
    main()
