"""GEMM epilogue activations of the bf16 engines against float64: GELU (BERT FFN1 forward, with the pre-activation
copy) and GELU' (the FFN2 input gradient) through the branch-free erf (common.h erf_fast, |error| <= 1.5e-7), and
the library-erff path (VCG_FAST_GELU=0 semantics are the same formula).

Exactness check: a GEMM with A = [x, 0...], B = e_0 computes gelu(x) of every bf16 value x in [-6, 6]; the bf16
output must be the correctly rounded float64 gelu(x) except where the value sits within 2e-7 (relative) of a bf16
rounding boundary. Tolerance for the full GEMMs: 2e-2 of max|ref| (bf16 operands, one output rounding)."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module")
def K():
    from vcg_hip import _lib, ops
    _lib.call("vcg_init", 0)
    return ops


def _gelu64(x):
    return 0.5 * x * (1.0 + torch.erf(x / 2 ** 0.5))


def test_gelu_epilogue_correctly_rounded(K):
    x = torch.linspace(-6, 6, 8192 * 4, dtype=torch.float64).to(torch.bfloat16).unique()
    M = (x.numel() + 127) // 128 * 128
    A = torch.zeros(M, 64, dtype=torch.bfloat16)
    A[:x.numel(), 0] = x
    B = torch.zeros(64, 64, dtype=torch.bfloat16)
    B[0, 0] = 1.0
    bias = torch.zeros(64, device=DEV)
    out = K.gemm(A.to(DEV), B.to(DEV), M, 64, 64, 64, 64, bias=bias, act=K.ACT_GELU)[:x.numel(), 0].double().cpu()
    ref = _gelu64(x.double())
    # erf's absolute error (1.5e-7, plus fp32 rounding) becomes 0.5 |x| 2.5e-7 in gelu: the output must be a bf16
    # neighbour of gelu(x) within that band (exactly the correctly rounded value away from rounding boundaries;
    # where 1 + erf cancels -- x << 0, gelu ~ 1e-8 -- the band is absolute, as it is for the library erff)
    band = 0.5 * x.double().abs() * 2.5e-7 + 1e-30
    lo = (ref - band).to(torch.bfloat16).double()
    hi = (ref + band).to(torch.bfloat16).double()
    ok = (out >= torch.minimum(lo, hi)) & (out <= torch.maximum(lo, hi))
    assert ok.all(), f"{int((~ok).sum())} GELU values outside the error band, e.g. x={x[~ok][:4].tolist()} " \
                     f"got {out[~ok][:4].tolist()} ref {ref[~ok][:4].tolist()}"
    exact = ref.to(torch.bfloat16).double()
    away = x.double() > -3.0  # (below, 1 + erf cancels and only the absolute band above holds)
    assert (out == exact)[away].double().mean().item() > 0.99


@pytest.mark.parametrize("M", [8192, 300])
def test_ffn_gelu_fwd_and_bwd(K, M):
    H, I = 768, 3072
    x = torch.randn(M, H).to(torch.bfloat16)
    W1 = (torch.randn(I, H) * 0.03).to(torch.bfloat16)
    b1 = torch.randn(I) * 0.1
    pre = torch.empty(M, I, dtype=torch.bfloat16, device=DEV)
    ff = K.gemm(x.to(DEV), W1.to(DEV), M, I, H, H, H, bias=b1.to(DEV), act=K.ACT_GELU, aux=pre)
    p64 = x.double() @ W1.double().T + b1.double()
    scale = p64.abs().max().item()
    assert (pre.double().cpu() - p64).abs().max().item() <= 2e-2 * scale
    g64 = _gelu64(p64)
    assert (ff.double().cpu() - g64).abs().max().item() <= 2e-2 * g64.abs().max().item()
    # FFN2 input gradient: dpre = (dfo @ W2) * gelu'(pre)
    W2 = (torch.randn(H, I) * 0.03).to(torch.bfloat16)
    dfo = torch.randn(M, H).to(torch.bfloat16)
    dpre = K.gemm(dfo.to(DEV), W2.to(DEV), M, I, H, H, I, transB=True, act=K.ACT_GELU_BWD, residual=pre, ldr=I)
    pr = pre.double().cpu()
    cdf = 0.5 * (1 + torch.erf(pr / 2 ** 0.5))
    d64 = (dfo.double() @ W2.double()) * (cdf + pr * torch.exp(-0.5 * pr * pr) / (2 * torch.pi) ** 0.5)
    assert (dpre.double().cpu() - d64).abs().max().item() <= 2e-2 * d64.abs().max().item()
    # the same with W2^T materialised (the BERT backward's B operand, _LinearT): the fast engine's staged GELU'
    # epilogue (dh rounded to bf16, then times GELU'(pre), full-row residual reads)
    W2t = W2.T.contiguous().to(DEV)
    dpre2 = K.gemm(dfo.to(DEV), W2t, M, I, H, H, H, act=K.ACT_GELU_BWD, residual=pre, ldr=I)
    assert (dpre2.double().cpu() - d64).abs().max().item() <= 2e-2 * d64.abs().max().item()
    dh = (dfo.to(DEV) @ W2.to(DEV)).double()  # the rounded dh (torch bf16 GEMM), then the fp64 GELU' product
    ref2 = (dh.cpu() * (cdf + pr * torch.exp(-0.5 * pr * pr) / (2 * torch.pi) ** 0.5))
    rel = (dpre2.double().cpu() - ref2).abs().max().item() / ref2.abs().max().item()
    assert rel <= 1e-2, rel
