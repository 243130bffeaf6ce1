"""Micro-benchmark of the BERT-base GEMMs at B=64 x L=128 (8192 token rows), bf16, HIP events: the wide-tile
engine (ops.ACT_FLAG_WIDE, the product path) against the 128 x 128 engine (the same call unflagged) and torch.matmul
(the vendor library, for the headroom estimate only -- never on the product path): forward projections (with the
GELU + pre-activation epilogue for FFN1), input-gradient GEMMs (W^T resident; FFN2's with the GELU' epilogue) and
weight-gradient split-K GEMMs.
Usage: python tools/bench_bert_gemm.py [--widths 128,192,256]"""
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
    return e0.elapsed_time(e1) / iters * 1e3  # us


def wide_line(name, fn, fl, widths):
    """Time fn on the wide engine at its default tile width and at each forced width."""
    out = []
    t = timeit(fn)
    out.append(f"{name} {t:7.1f}us {fl / t / 1e6:6.0f}TF/s")
    for w in widths:
        os.environ["VCG_WIDE_BN"] = str(w)
        t = timeit(fn)
        out.append(f"[{w}: {t:6.1f}us {fl / t / 1e6:5.0f}]")
    os.environ.pop("VCG_WIDE_BN", None)
    return "  ".join(out)


def main():
    dt, dev = torch.bfloat16, "cuda"
    widths = [int(w) for w in sys.argv[sys.argv.index("--widths") + 1].split(",")] if "--widths" in sys.argv else []
    print("torch blas:", torch.backends.cuda.preferred_blas_library(), flush=True)
    W_ = ops.ACT_FLAG_WIDE
    R, H, I = 8192, 768, 3072
    x = torch.randn(R, H, device=dev).to(dt)
    xi = torch.randn(R, I, device=dev).to(dt)
    for (N, K, name) in ((3 * H, H, "qkv"), (H, H, "out-proj"), (I, H, "ffn1"), (H, I, "ffn2")):
        W = (torch.randn(N, K, device=dev) * 0.02).to(dt)
        b = torch.zeros(N, device=dev)
        A = x if K == H else xi
        fl = 2.0 * R * N * K
        print(f"{name:9s} " + wide_line("WIDE fwd", lambda: ops.gemm(A, W, R, N, K, K, K, bias=b, act=W_), fl, widths),
              flush=True)
        if name == "ffn1":
            pre = torch.empty(R, N, dtype=dt, device=dev)
            print(f"{name:9s} " + wide_line("WIDE gelu+aux", lambda: ops.gemm(A, W, R, N, K, K, K, bias=b,
                                                                              act=ops.ACT_GELU | W_, aux=pre), fl, widths),
                  flush=True)
        dY = torch.randn(R, N, device=dev).to(dt)
        Wt = ops.transpose(W)
        if name == "ffn2":
            pre = torch.randn(R, K, device=dev).to(dt)
            print(f"{name:9s} " + wide_line("WIDE dX+gelu'", lambda: ops.gemm(dY, Wt, R, K, N, N, N,
                                                                              act=ops.ACT_GELU_BWD | W_, residual=pre,
                                                                              ldr=K), fl, widths), flush=True)
        rK = torch.randn(R, K, device=dev).to(dt)
        print(f"{name:9s} " + wide_line("WIDE dX+res", lambda: ops.gemm(dY, Wt, R, K, N, N, N, residual=rK, ldr=K,
                                                                        act=W_), fl, widths), flush=True)
        t = timeit(lambda: ops.gemm(A, W, R, N, K, K, K, bias=b))
        line = [f"{name:9s} fwd {t:7.1f}us {fl / t / 1e6:6.0f}TF/s"]
        # (the vendor library on the same shape, for the headroom estimate only -- never on the product path)
        t = timeit(lambda: torch.matmul(A, W.t()))
        line.append(f"[hipBLASLt {t:7.1f}us {fl / t / 1e6:6.0f}TF/s]")
        if name == "ffn1":
            pre = torch.empty(R, N, dtype=dt, device=dev)
            t = timeit(lambda: ops.gemm(A, W, R, N, K, K, K, bias=b, act=ops.ACT_GELU, aux=pre))
            line.append(f"gelu+aux {t:7.1f}us {fl / t / 1e6:6.0f}TF/s")
            t = timeit(lambda: ops.gemm(A, W, R, N, K, K, K, bias=b, act=ops.ACT_GELU))
            line.append(f"gelu {t:7.1f}us")
            t = timeit(lambda: ops.gemm(A, W, R, N, K, K, K, bias=b, act=ops.ACT_RELU))
            line.append(f"relu {t:7.1f}us")
        # input gradient: dA [R, K] = dY [R, N] @ W [N, K]
        dY = torch.randn(R, N, device=dev).to(dt)
        t = timeit(lambda: ops.gemm(dY, W, R, K, N, N, K, transB=True))
        line.append(f"dX transB {t:7.1f}us {fl / t / 1e6:6.0f}TF/s")
        if name == "ffn2":  # the FFN2 input gradient carries the GELU derivative of the saved pre-activation
            pre = torch.randn(R, K, device=dev).to(dt)
            t = timeit(lambda: ops.gemm(dY, W, R, K, N, N, K, transB=True, act=ops.ACT_GELU_BWD, residual=pre, ldr=K))
            line.append(f"dX transB+gelu' {t:7.1f}us")
            t = timeit(lambda: ops.gemm(dY, ops.transpose(W), R, K, N, N, N, act=ops.ACT_GELU_BWD, residual=pre, ldr=K))
            line.append(f"dX W^T+gelu' {t:7.1f}us")
            Wt = ops.transpose(W)
            t = timeit(lambda: ops.gemm(dY, Wt, R, K, N, N, N, act=ops.ACT_GELU_BWD, residual=pre, ldr=K))
            line.append(f"dX (W^T resident)+gelu' {t:7.1f}us {fl / t / 1e6:6.0f}TF/s")
        t = timeit(lambda: ops.gemm(dY, ops.transpose(W), R, K, N, N, N))
        line.append(f"dX W^T {t:7.1f}us {fl / t / 1e6:6.0f}TF/s")
        t = timeit(lambda: torch.matmul(dY, W))
        line.append(f"[lib dX {t:7.1f}us {fl / t / 1e6:6.0f}TF/s]")
        t = timeit(lambda: torch.matmul(dY.t(), A))
        line.append(f"[lib dW {t:7.1f}us {fl / t / 1e6:6.0f}TF/s]")
        t = timeit(lambda: ops.transpose(W))
        line.append(f"(transpose {t:5.1f}us)")
        gW = torch.zeros(N, K, device=dev)
        wsb = ops.gemm_splitk(dY, A, gW, N, K, R, N, K, transA=True, transB=True)
        t = timeit(lambda: ops.gemm_splitk(dY, A, gW, N, K, R, N, K, transA=True, transB=True, workspace=wsb))
        line.append(f"dW {t:7.1f}us {fl / t / 1e6:6.0f}TF/s")
        print("  ".join(line), flush=True)


if __name__ == "__main__":
    main()
