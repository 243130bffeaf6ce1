"""BERT-base's plain GEMMs on the vendor library (csrc/blaslt.hip, through vcg_gemm / vcg_gemm_splitk) against the
hand-written engine (VCG_LT_GEMM=0) and a float64 reference of the same product: the projections' forward with a
bias, the input gradients with and without a residual addend (W^T resident and transposed-B forms), and the weight
gradients into an fp32 gradient with and without accumulation (opt-in, VCG_LT_DW=1), and FFN1 as the library GEMM
plus a GELU pass, at the B = 64 x L = 128 shapes of the bench. Both
paths sit within bf16 output rounding of float64 (the library's error no larger than 1.5x the engine's + a bf16
ulp), the library path is deterministic (bit-identical repeat), and a GEMM below the size threshold or with a
fused activation other than FFN1's GELU stays on the engine (bit-identical with and without the library)."""
import pytest
import torch

from vcg_hip import _lib, ops

pytestmark = pytest.mark.gpu
DEV = "cuda"
R, H, I = 8192, 768, 3072
LIB = ops.ACT_FLAG_LIB


@pytest.fixture(scope="module", autouse=True)
def _init():
    _lib.call("vcg_init", 0)


def _bf(shape, gen, scale=1.0):
    return (torch.randn(*shape, generator=gen) * scale).to(torch.bfloat16).to(DEV)


def _rel(a, ref):
    return ((a.double() - ref).norm() / ref.norm()).item()


def _both(monkeypatch, fn):
    out = {}
    for flag in ("1", "0"):
        monkeypatch.setenv("VCG_LT_GEMM", flag)
        out[flag] = fn()
        torch.cuda.synchronize()
    monkeypatch.delenv("VCG_LT_GEMM")
    return out["1"], out["0"]


@pytest.mark.parametrize("N,K", [(3 * H, H), (H, H), (I, H), (H, I)])
def test_forward_bias(monkeypatch, N, K):
    gen = torch.Generator().manual_seed(N + K)
    A, W = _bf((R, K), gen), _bf((N, K), gen, 0.02)
    b = (torch.randn(N, generator=gen) * 0.1).to(DEV)
    lt, eng = _both(monkeypatch, lambda: ops.gemm(A, W, R, N, K, K, K, bias=b, act=LIB))
    ref = A.double() @ W.double().t() + b.double()
    e_lt, e_eng = _rel(lt, ref), _rel(eng, ref)
    print(f"fwd N={N} K={K}: lib {e_lt:.2e} engine {e_eng:.2e}")
    assert e_lt < 1.5 * e_eng + 4e-3
    again = ops.gemm(A, W, R, N, K, K, K, bias=b, act=LIB)
    torch.cuda.synchronize()
    assert torch.equal(lt, again)


@pytest.mark.parametrize("N,K,res,wt", [(H, I, True, True), (H, 3 * H, True, True), (H, H, False, False),
                                        (H, H, True, False)])
def test_input_gradient(monkeypatch, N, K, res, wt):
    """dX [R, N] = dY [R, K] @ W [K, N] (+ residual): W^T resident ([N][K], the engine's form for long K) or the
    transposed-B form over W [K][N]."""
    gen = torch.Generator().manual_seed(N * 3 + K)
    dY, W = _bf((R, K), gen, 0.05), _bf((K, N), gen, 0.02)
    r = _bf((R, N), gen, 0.01) if res else None
    Wt = W.t().contiguous()
    if wt:
        fn = lambda: ops.gemm(dY, Wt, R, N, K, K, K, residual=r, ldr=N, act=LIB)  # noqa: E731
    else:
        fn = lambda: ops.gemm(dY, W, R, N, K, K, N, transB=True, residual=r, ldr=N, act=LIB)  # noqa: E731
    lt, eng = _both(monkeypatch, fn)
    ref = dY.double() @ W.double() + (r.double() if res else 0.0)
    e_lt, e_eng = _rel(lt, ref), _rel(eng, ref)
    print(f"dX N={N} K={K} res={res} wt={wt}: lib {e_lt:.2e} engine {e_eng:.2e}")
    assert e_lt < 1.5 * e_eng + 4e-3


@pytest.mark.parametrize("M,N,acc", [(H, I, True), (I, H, False), (3 * H, H, True), (H, H, True)])
def test_weight_gradient(monkeypatch, M, N, acc):
    """gW [M, N] (+)= dY^T [M, R] @ X [R, N] into fp32 (gemm_splitk, transA / transB)."""
    gen = torch.Generator().manual_seed(M + 7 * N)
    dY, X = _bf((R, M), gen, 0.05), _bf((R, N), gen)
    g0 = torch.randn(M, N, generator=gen).to(DEV) * 0.1

    def run():
        g = g0.clone()
        ops.gemm_splitk(dY, X, g, M, N, R, M, N, transA=True, transB=True, accumulate=acc)
        return g
    lt, eng = _both(monkeypatch, run)
    ref = dY.double().t() @ X.double() + (g0.double() if acc else 0.0)
    e_lt, e_eng = _rel(lt, ref), _rel(eng, ref)
    print(f"dW M={M} N={N} acc={acc}: lib {e_lt:.2e} engine {e_eng:.2e}")
    assert e_lt < 1e-5 and e_eng < 1e-5
    assert torch.equal(lt, run())


def test_small_and_fused_stay_on_engine(monkeypatch):
    """Below the size threshold (the pooler, B = 64 rows) and with a fused activation (GELU + pre-activation) the
    engine runs either way: bit-identical with and without the library."""
    gen = torch.Generator().manual_seed(5)
    A, W = _bf((64, H), gen), _bf((H, H), gen, 0.02)
    b = torch.randn(H, generator=gen).to(DEV) * 0.1
    lt, eng = _both(monkeypatch, lambda: ops.gemm(A, W, 64, H, H, H, H, bias=b, act=ops.ACT_TANH | LIB))
    assert torch.equal(lt, eng)
    A2, W2 = _bf((R, H), gen), _bf((I, H), gen, 0.02)
    b2 = torch.randn(I, generator=gen).to(DEV) * 0.1

    def ffn1():
        p = torch.empty((R, I), dtype=torch.bfloat16, device=DEV)
        o = ops.gemm(A2, W2, R, I, H, H, H, bias=b2, act=ops.ACT_GELU | LIB, aux=p)
        return torch.cat([o, p])
    monkeypatch.setenv("VCG_LT_GELU_OFF", "1")
    lt, eng = _both(monkeypatch, ffn1)
    assert torch.equal(lt, eng)


def test_ffn1_gelu_library_plus_pass(monkeypatch):
    """FFN1 on the library: pre = bf16(x W^T + b), then ff = bf16(gelu(pre)) in a separate pass (the reference's
    bf16-autocast order: Linear -> GELU on the rounded pre-activation). pre within bf16 rounding of float64, ff equal
    to a torch GELU (erf) of the stored pre within one bf16 ulp, both within bf16 rounding of the engine's fused
    epilogue (which applies GELU to the fp32 pre-activation)."""
    gen = torch.Generator().manual_seed(6)
    A, W = _bf((R, H), gen), _bf((I, H), gen, 0.05)
    b = torch.randn(I, generator=gen).to(DEV) * 0.1

    def ffn1():
        p = torch.empty((R, I), dtype=torch.bfloat16, device=DEV)
        o = ops.gemm(A, W, R, I, H, H, H, bias=b, act=ops.ACT_GELU | LIB, aux=p)
        return o, p
    (o_lt, p_lt), (o_en, p_en) = _both(monkeypatch, ffn1)
    ref = A.double() @ W.double().t() + b.double()
    assert _rel(p_lt, ref) < 4e-3 and _rel(p_en, ref) < 4e-3
    g = torch.nn.functional.gelu(p_lt.float()).to(torch.bfloat16)
    d = (o_lt.float() - g.float()).abs()
    assert (d <= 2 ** -7 * g.float().abs().clamp_min(2 ** -10)).all()
    gref = torch.nn.functional.gelu(ref)
    assert _rel(o_lt, gref) < 6e-3 and _rel(o_en, gref) < 6e-3
    o2, p2 = ffn1()
    torch.cuda.synchronize()
    assert torch.equal(o2, o_lt) and torch.equal(p2, p_lt)


def test_without_flag_stays_on_engine(monkeypatch):
    """A GEMM without ops.ACT_FLAG_LIB (every trunk GEMM) runs on the engine whatever its shape: bit-identical with
    the library on and off."""
    gen = torch.Generator().manual_seed(7)
    A, W = _bf((R, H), gen), _bf((I, H), gen, 0.02)
    b = torch.randn(I, generator=gen).to(DEV) * 0.1
    lt, eng = _both(monkeypatch, lambda: ops.gemm(A, W, R, I, H, H, H, bias=b))
    assert torch.equal(lt, eng)


@pytest.mark.parametrize("M,N,K,pad", [(8255, 2304, 768, 64), (9000, 768, 3072, 0), (6400, 3072, 768, 8)])
def test_ragged_rows_and_pitch(monkeypatch, M, N, K, pad):
    """Row counts that are not a multiple of any tile (B x L of other batch / sequence sizes) and an output row pitch
    wider than N (a view into a wider buffer): the library writes exactly the M x N block -- the padding columns keep
    their sentinel -- within bf16 rounding of float64, with the bias and with a residual of the same pitch."""
    gen = torch.Generator().manual_seed(M + N + K)
    A, W = _bf((M, K), gen), _bf((N, K), gen, 0.02)
    b = (torch.randn(N, generator=gen) * 0.1).to(DEV)
    ld = N + pad
    r = _bf((M, ld), gen, 0.01)

    def run(res):
        buf = torch.full((M, ld), 7.0, dtype=torch.bfloat16, device=DEV)
        out = buf[:, :N]
        if res:
            ops.gemm(A, W, M, N, K, K, K, out=out, ldc=ld, residual=r, ldr=ld, act=LIB)
        else:
            ops.gemm(A, W, M, N, K, K, K, out=out, ldc=ld, bias=b, act=LIB)
        return buf
    for res in (False, True):
        lt, eng = _both(monkeypatch, lambda: run(res))
        ref = A.double() @ W.double().t() + (r[:, :N].double() if res else b.double())
        assert _rel(lt[:, :N], ref) < 1.5 * _rel(eng[:, :N], ref) + 4e-3
        if pad:
            assert (lt[:, N:] == 7.0).all()
