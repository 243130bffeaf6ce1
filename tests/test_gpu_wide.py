"""The wide-tile GEMM engine (csrc/igemm_wide.hip, vcg_gemm with VCG_ACT_FLAG_WIDE) on BERT-base's Linear layers
(reference: transformers BertModel's nn.Linear, model/lang/bert_hugface.py:20) and the trunk's downsample input
gradient, against a float64 reference of the same product and against the 128 x 128 engine (the same call without
the flag):
  * every epilogue class -- bias, bias + GELU with the pre-activation, GELU' of the pre-activation, residual addend --
    at the B = 64 x L = 128 shapes of the bench (8192 rows), and at B = 1 (128 rows: the oracle-anchored step);
  * all three tile widths (128 / 192 / 256 columns), ragged M / N / K, pitched outputs, no bias;
  * within bf16 output rounding of float64 (no worse than the 128 x 128 engine + a bf16 ulp), deterministic
    (bit-identical repeat), and the census names the kernel that ran.
GELU follows bf16 autocast: GELU of the bf16-rounded pre-activation."""
import math

import pytest
import torch

from vcg_hip import _lib, ops

pytestmark = pytest.mark.gpu
DEV = "cuda"
R, H, I = 8192, 768, 3072
WIDE = ops.ACT_FLAG_WIDE


@pytest.fixture(scope="module", autouse=True)
def _init():
    _lib.call("vcg_init", 0)


def _bf(shape, gen, scale=1.0):
    return (torch.randn(*shape, generator=gen) * scale).to(torch.bfloat16).to(DEV)


def _rel(a, ref):
    return ((a.double() - ref).norm() / ref.norm()).item()


def _gelu64(x):
    return 0.5 * x * (1.0 + torch.erf(x / math.sqrt(2.0)))


def _gelu_grad64(x):
    return 0.5 * (1.0 + torch.erf(x / math.sqrt(2.0))) + x * torch.exp(-0.5 * x * x) / math.sqrt(2.0 * math.pi)


def _wide(fn):
    """Run fn with the census on; return (result, census keys of gemm_wide launches)."""
    ops.gemm_census_enable(True)
    out = fn()
    torch.cuda.synchronize()
    keys = [k for k in ops.gemm_census() if k.startswith("gemm_wide")]
    ops.gemm_census_enable(False)
    return out, keys


@pytest.mark.parametrize("M", [R, 128])
@pytest.mark.parametrize("N,K", [(3 * H, H), (H, H), (I, H), (H, I)])
def test_forward_bias(M, N, K):
    gen = torch.Generator().manual_seed(N + K + M)
    A, W = _bf((M, K), gen), _bf((N, K), gen, 0.02)
    b = (torch.randn(N, generator=gen) * 0.1).to(DEV)
    wide, keys = _wide(lambda: ops.gemm(A, W, M, N, K, K, K, bias=b, act=WIDE))
    assert keys and all(f"M={M} N={N} K={K}" in k for k in keys), keys
    eng = ops.gemm(A, W, M, N, K, K, K, bias=b)
    ref = A.double() @ W.double().t() + b.double()
    e_w, e_e = _rel(wide, ref), _rel(eng, ref)
    print(f"fwd M={M} N={N} K={K} {keys}: wide {e_w:.2e} engine {e_e:.2e}")
    assert e_w < 1.5 * e_e + 4e-3
    again = ops.gemm(A, W, M, N, K, K, K, bias=b, act=WIDE)
    torch.cuda.synchronize()
    assert torch.equal(wide, again)


@pytest.mark.parametrize("M", [R, 128])
def test_ffn1_gelu_aux(M):
    """pre = bf16(x W^T + b) (the pre-activation the backward keeps), out = bf16(gelu(x W^T + b)) of the unrounded
    value: pre within bf16 rounding of float64, out equal to the float64 GELU of the exact pre-activation within bf16
    rounding, and to the 128 x 128 engine's fused epilogue within one bf16 ulp."""
    gen = torch.Generator().manual_seed(11 + M)
    A, W = _bf((M, H), gen), _bf((I, H), gen, 0.02)
    b = (torch.randn(I, generator=gen) * 0.1).to(DEV)
    pre = torch.empty((M, I), dtype=torch.bfloat16, device=DEV)
    out, keys = _wide(lambda: ops.gemm(A, W, M, I, H, H, H, bias=b, act=ops.ACT_GELU | WIDE, aux=pre))
    assert keys and "we1" in keys[0], keys
    ref_pre = A.double() @ W.double().t() + b.double()
    assert _rel(pre, ref_pre) < 4e-3
    g = _gelu64(ref_pre)
    assert _rel(out, g) < 4e-3
    eng = ops.gemm(A, W, M, I, H, H, H, bias=b, act=ops.ACT_GELU)
    err = (out.double() - eng.double()).abs()
    assert (err <= eng.double().abs() * 2.0 ** -7 + 1e-6).all(), err.max().item()
    # no pre-activation copy: the same output
    out2 = ops.gemm(A, W, M, I, H, H, H, bias=b, act=ops.ACT_GELU | WIDE)
    torch.cuda.synchronize()
    assert torch.equal(out, out2)


@pytest.mark.parametrize("M", [R, 128])
def test_ffn2_input_gradient_gelu_bwd(M):
    """dpre = bf16(bf16(dY W) * gelu'(pre)) (FFN2's input gradient through the GELU, W^T resident)."""
    gen = torch.Generator().manual_seed(23 + M)
    dY, Wt = _bf((M, H), gen, 0.05), _bf((I, H), gen, 0.02)  # Wt = FFN2 weight^T [I][H]: K-contiguous
    pre = _bf((M, I), gen)
    out, keys = _wide(lambda: ops.gemm(dY, Wt, M, I, H, H, H, act=ops.ACT_GELU_BWD | WIDE, residual=pre, ldr=I))
    assert keys and "we2" in keys[0], keys
    eng = ops.gemm(dY, Wt, M, I, H, H, H, act=ops.ACT_GELU_BWD, residual=pre, ldr=I)
    ref = (dY.double() @ Wt.double().t()) * _gelu_grad64(pre.double())
    e_w, e_e = _rel(out, ref), _rel(eng, ref)
    print(f"gelu' M={M}: wide {e_w:.2e} engine {e_e:.2e}")
    assert e_w < 1.5 * e_e + 4e-3


@pytest.mark.parametrize("M", [R, 128])
@pytest.mark.parametrize("N,K", [(H, I), (H, 3 * H), (H, H)])
def test_input_gradient_residual(M, N, K):
    """dX [M, N] = dY [M, K] @ W^T-resident [N, K]^T + residual (the QKV / FFN1 input gradients add the skip branch)."""
    gen = torch.Generator().manual_seed(N * 3 + K + M)
    dY, Wt = _bf((M, K), gen, 0.05), _bf((N, K), gen, 0.02)
    r = _bf((M, N), gen, 0.01)
    out, keys = _wide(lambda: ops.gemm(dY, Wt, M, N, K, K, K, residual=r, ldr=N, act=WIDE))
    assert keys and "we3" in keys[0], keys
    eng = ops.gemm(dY, Wt, M, N, K, K, K, residual=r, ldr=N)
    ref = dY.double() @ Wt.double().t() + r.double()
    e_w, e_e = _rel(out, ref), _rel(eng, ref)
    print(f"dX M={M} N={N} K={K}: wide {e_w:.2e} engine {e_e:.2e}")
    assert e_w < 1.5 * e_e + 4e-3


@pytest.mark.parametrize("M", [R, 128])
@pytest.mark.parametrize("N,K", [(H, I), (H, 3 * H)])
def test_input_gradient_fp32_stream(M, N, K):
    """dX + the fp32 residual-gradient stream, written fp32 (VCG_ACT_FLAG_F32_OUT): within fp32 rounding of
    (bf16 operands' exact product + residual), i.e. far inside the bf16-output error."""
    gen = torch.Generator().manual_seed(N + K + 5 * M)
    dY, Wt = _bf((M, K), gen, 0.05), _bf((N, K), gen, 0.02)
    r = (torch.randn(M, N, generator=gen) * 0.01).to(DEV)
    out = torch.empty((M, N), dtype=torch.float32, device=DEV)
    _, keys = _wide(lambda: ops.gemm(dY, Wt, M, N, K, K, K, out=out, ldc=N, residual=r, ldr=N,
                                     act=WIDE | ops.ACT_FLAG_F32_OUT))
    assert keys and "we4" in keys[0], keys
    ref = dY.double() @ Wt.double().t() + r.double()
    assert _rel(out, ref) < 1e-5
    with pytest.raises(Exception):  # only with the wide flag and a residual
        ops.gemm(dY, Wt, M, N, K, K, K, out=out, ldc=N, act=ops.ACT_FLAG_F32_OUT)


@pytest.mark.parametrize("bn", ["128", "192", "256"])
@pytest.mark.parametrize("M,N,K", [(1000, 200, 136), (130, 776, 72), (1, 8, 8), (4099, 1032, 520)])
def test_ragged_all_widths(monkeypatch, bn, M, N, K):
    """Ragged M / N / K on every tile width (rows / columns beyond the matrix zero-filled by the loader and not
    stored), no bias, a pitched output (ldc > N) whose padding columns stay untouched."""
    monkeypatch.setenv("VCG_WIDE_BN", bn)
    gen = torch.Generator().manual_seed(M + N + K)
    A, W = _bf((M, K), gen), _bf((N, K), gen, 0.1)
    ld = N + 24
    out = torch.full((M, ld), 7.0, dtype=torch.bfloat16, device=DEV)
    _, keys = _wide(lambda: ops.gemm(A, W, M, N, K, K, K, out=out, ldc=ld, act=WIDE))
    assert keys and keys[0].startswith(f"gemm_wide 128x{bn} "), keys
    ref = A.double() @ W.double().t()
    assert _rel(out[:, :N], ref) < 4e-3
    assert (out[:, N:] == 7.0).all()
    r = _bf((M, N), gen, 0.5)
    o2 = ops.gemm(A, W, M, N, K, K, K, residual=r, ldr=N, act=WIDE)
    assert _rel(o2, ref + r.double()) < 4e-3


@pytest.mark.parametrize("M", [R, 128, 1])
def test_tile_width_choice(M):
    """The tile width follows N alone (192 columns at N = 768 / 2304, 256 at N = 3072, 128 at the downsample's 256 /
    512 / 1024), the same at every M."""
    gen = torch.Generator().manual_seed(3)
    A = _bf((M, H), gen)
    for N, bn in ((H, 192), (3 * H, 192), (I, 256), (256, 128), (512, 128), (1024, 128)):
        W = _bf((N, H), gen, 0.02)
        _, keys = _wide(lambda: ops.gemm(A, W, M, N, H, H, H, act=WIDE))
        assert keys == [f"gemm_wide 128x{bn} we0 M={M} N={N} K={H}"], keys


def test_unflagged_and_fp32_stay_off():
    """Without the flag, with transposed operands, or in fp32 the wide engine does not run."""
    gen = torch.Generator().manual_seed(9)
    A, W = _bf((256, 128), gen), _bf((128, 128), gen)
    _, keys = _wide(lambda: ops.gemm(A, W, 256, 128, 128, 128, 128))
    assert keys == []
    _, keys = _wide(lambda: ops.gemm(A, W, 256, 128, 128, 128, 128, transB=True, act=WIDE))
    assert keys == []
    Af, Wf = A.float(), W.float()
    _, keys = _wide(lambda: ops.gemm(Af, Wf, 256, 128, 128, 128, 128, act=WIDE))
    assert keys == []
