"""Per-kernel numerics of libvcg_hip against plain fp64 torch references of the same op.

fp32 storage (MFMA f32 16x16x4): relative error ~1e-6; bf16 storage (MFMA bf16 16x16x32,
fp32 accumulate): inputs are rounded to bf16 first, tolerance 2e-2 relative to max|ref|
(one bf16 output rounding is 2^-8).
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

DEV = "cuda"
DTYPES = [torch.float32, torch.bfloat16]


def _tol(dtype):
    return 2e-5 if dtype == torch.float32 else 2e-2


def _close(out, ref, dtype, what=""):
    out = out.detach().double().cpu()
    ref = ref.detach().double().cpu()
    scale = ref.abs().max().item() + 1e-6
    err = (out - ref).abs().max().item()
    assert err <= _tol(dtype) * scale, f"{what}: max err {err:.3e} vs scale {scale:.3e}"


def _rand(shape, dtype, seed, scale=1.0):
    g = torch.Generator().manual_seed(seed)
    x = (torch.randn(shape, generator=g) * scale).to(dtype)
    return x


def tsm_ref(x, T, fold):
    """Reference TemporalShift.shift (ops/temporal_shift.py:33-51) on NCHW."""
    nt, c, h, w = x.shape
    x = x.view(nt // T, T, c, h, w)
    out = torch.zeros_like(x)
    out[:, :-1, :fold] = x[:, 1:, :fold]
    out[:, 1:, fold:2 * fold] = x[:, :-1, fold:2 * fold]
    out[:, :, 2 * fold:] = x[:, :, 2 * fold:]
    return out.view(nt, c, h, w)


@pytest.fixture(scope="module")
def K():
    from vcg_hip import ops, _lib
    _lib.call("vcg_init", 0)
    return ops


def test_synth_bitexact(K):
    from vcg_hip import synth
    for kind, a, b in [(0, -0.5, 2.0), (1, 0.1, 0.02), (2, 1000, 30522)]:
        n = 100003
        dt = torch.int64 if kind == 2 else torch.float32
        t = torch.empty(n, dtype=dt, device=DEV)
        K.synth(t, kind, 0x1234567, a, b)
        ref = synth.fill_np(n, kind, 0x1234567, a, b)
        assert np.array_equal(t.cpu().numpy(), ref), f"kind {kind} not bit-exact"


CONV_CASES = [
    # N, H, W, Cin, Cout, KH, stride, pad, tsm_T
    (4, 8, 8, 64, 64, 1, 1, 0, 0),
    (4, 8, 8, 64, 128, 3, 1, 1, 0),
    (4, 9, 9, 64, 128, 3, 2, 1, 0),
    (4, 8, 8, 64, 256, 1, 2, 0, 0),
    (8, 6, 6, 64, 64, 1, 1, 0, 4),
    (8, 5, 7, 128, 64, 1, 1, 0, 4),
    (2, 16, 16, 3, 64, 7, 2, 3, 0),  # stem
]


def _prep(K, x_nchw, w, dtype, T, fold):
    N, C, H, W = x_nchw.shape
    cpad = C if C >= 8 else (8 if dtype == torch.bfloat16 else 4)
    xs = torch.zeros((N, H, W, cpad), dtype=dtype)
    xs[..., :C] = x_nchw.permute(0, 2, 3, 1).to(dtype)
    return xs.to(DEV), cpad


@pytest.mark.parametrize("dtype", DTYPES)
@pytest.mark.parametrize("case", CONV_CASES)
def test_conv_fwd_and_stats(K, dtype, case):
    N, H, W, Cin, Cout, KH, s, p, T = case
    x = _rand((N, Cin, H, W), dtype, 1).double()
    w = _rand((Cout, Cin, KH, KH), torch.float32, 2, 0.1)
    fold = Cin // 8 if T else 0
    xin = tsm_ref(x, T, fold) if T else x
    ref = F.conv2d(xin, w.to(dtype).double(), stride=s, padding=p)  # NCHW
    xs, cpad = _prep(K, x, w, dtype, T, fold)
    wd = K.weight_prep(w.to(DEV), cpad, dtype)
    OH, OW = ref.shape[2], ref.shape[3]
    M = N * OH * OW
    mt = K.stats_tiles(M)
    stats = K.stats_buffer(Cout, M, DEV)
    y = K.conv_fwd(xs, wd, N, H, W, cpad, Cout, KH, KH, s, p, T, fold, stats=stats)
    _close(y.permute(0, 3, 1, 2), ref, dtype, "conv fwd")
    # BN statistics of the stored output
    yref = y.double().cpu().reshape(M, Cout)
    mean = torch.empty(Cout, device=DEV)
    invstd = torch.empty_like(mean)
    scale = torch.empty_like(mean)
    shift = torch.empty_like(mean)
    gamma = torch.rand(Cout, device=DEV) + 0.5
    beta = torch.randn(Cout, device=DEV)
    rm = torch.zeros(Cout, device=DEV)
    rv = torch.ones(Cout, device=DEV)
    K.bn_finalize(stats, mt, M, Cout, gamma, beta, mean, invstd, scale, shift, rm, rv, 0.1, 1e-5)
    torch.cuda.synchronize()
    mu = yref.mean(0)
    var = yref.var(0, unbiased=False)
    assert torch.allclose(mean.double().cpu(), mu, atol=1e-5 * (1 + mu.abs().max().item()))
    assert torch.allclose(invstd.double().cpu(), 1 / torch.sqrt(var + 1e-5), rtol=1e-4)
    assert torch.allclose(rv.double().cpu(), 0.9 + 0.1 * yref.var(0, unbiased=True), rtol=1e-4)


@pytest.mark.parametrize("case", [(16, 56, 56, 64, 256, 1, 1, 0, 0, 2.0), (8, 28, 28, 128, 128, 3, 1, 1, 0, 0.0),
                                  (8, 29, 27, 64, 64, 3, 1, 1, 4, 3.0),
                                  # >= 64 Ki rows
                                  (24, 56, 56, 64, 256, 1, 1, 0, 0, 2.0), (16, 65, 71, 64, 128, 3, 1, 1, 4, 1.0)])
def test_conv_stats_multitile(K, case):
    """BN statistics when persistent workgroups walk several M-tiles (one stats slot per workgroup
    row, count row), M not a multiple of 128, and outputs with |mean| >> std (shifted sums)."""
    N, H, W, Cin, Cout, KH, s, p, T, off = case
    dtype = torch.bfloat16
    x = (_rand((N, Cin, H, W), dtype, 5).double() + off).to(dtype).double()
    w = (_rand((Cout, Cin, KH, KH), torch.float32, 6, 0.05) + 0.02).to(dtype)
    fold = Cin // 8 if T else 0
    xs, cpad = _prep(K, x, w, dtype, T, fold)
    wd = K.weight_prep(w.float().to(DEV), cpad, dtype)
    OH, OW = K.conv_out_hw(H, W, KH, KH, s, p)
    M = N * OH * OW
    stats = K.stats_buffer(Cout, M, DEV)
    y = K.conv_fwd(xs, wd, N, H, W, cpad, Cout, KH, KH, s, p, T, fold, stats=stats)
    z = torch.empty(Cout, device=DEV)
    mean, invstd, scale, shift = (torch.empty_like(z) for _ in range(4))
    K.bn_finalize(stats, K.stats_tiles(M), M, Cout, None, None, mean, invstd, scale, shift, None, None, 0.1, 1e-5)
    torch.cuda.synchronize()
    if M >= 65536:  # the 256-row kernel's output values too
        xin = tsm_ref(x, T, fold) if T else x
        ref = F.conv2d(xin, w.double(), stride=s, padding=p)
        _close(y.permute(0, 3, 1, 2), ref, dtype, "conv fwd (>= 64 Ki rows)")
    yref = y.double().cpu().reshape(M, Cout)
    mu, var = yref.mean(0), yref.var(0, unbiased=False)
    assert float(stats[Cout, :, 0].sum()) == M                      # slot row counts cover every row
    assert torch.allclose(mean.double().cpu(), mu, rtol=1e-5, atol=1e-5)
    assert torch.allclose(invstd.double().cpu(), 1 / torch.sqrt(var + 1e-5), rtol=2e-4)


@pytest.mark.parametrize("dtype", DTYPES)
@pytest.mark.parametrize("case", [c for c in CONV_CASES if c[3] >= 64])
def test_conv_dgrad(K, dtype, case):
    N, H, W, Cin, Cout, KH, s, p, T = case
    x = _rand((N, Cin, H, W), torch.float32, 3).double().requires_grad_()
    w = _rand((Cout, Cin, KH, KH), torch.float32, 4, 0.1)
    y = F.conv2d(x, w.to(dtype).double(), stride=s, padding=p)
    dy = _rand(y.shape, dtype, 5).double()
    (ref,) = torch.autograd.grad(y, x, dy)
    dys = dy.permute(0, 2, 3, 1).contiguous().to(dtype).to(DEV)
    wt = K.weight_prep(w.to(DEV), Cin, dtype, transposed=True)
    dx = K.conv_dgrad(dys, wt, N, H, W, Cin, Cout, KH, KH, s, p)
    _close(dx.permute(0, 3, 1, 2), ref, dtype, "conv dgrad")


@pytest.mark.parametrize("dtype", DTYPES)
@pytest.mark.parametrize("case", CONV_CASES)
def test_conv_wgrad(K, dtype, case):
    N, H, W, Cin, Cout, KH, s, p, T = case
    x = _rand((N, Cin, H, W), dtype, 6).double()
    fold = Cin // 8 if T else 0
    w = _rand((Cout, Cin, KH, KH), torch.float32, 7, 0.1).double().requires_grad_()
    xin = tsm_ref(x, T, fold) if T else x
    y = F.conv2d(xin, w, stride=s, padding=p)
    dy = _rand(y.shape, dtype, 8).double()
    (ref,) = torch.autograd.grad(y, w, dy)
    xs, cpad = _prep(K, x, None, dtype, T, fold)
    dys = dy.permute(0, 2, 3, 1).contiguous().to(dtype).to(DEV)
    dw = torch.full((Cout, Cin, KH, KH), 0.5, dtype=torch.float32, device=DEV)  # accumulate onto 0.5
    K.conv_wgrad(xs, dys, dw, N, H, W, cpad, Cin, Cout, KH, KH, s, p, T, fold, accumulate=True)
    _close(dw - 0.5, ref, dtype, "conv wgrad")


@pytest.mark.parametrize("case", [(2, 16, 16, 7, 2, 3), (3, 17, 22, 7, 2, 3), (4, 64, 64, 7, 2, 3),
                                  (2, 15, 12, 5, 2, 2), (2, 12, 14, 3, 2, 1)])
def test_stem_pair(K, case):
    """The pair-packed bf16 stem (C = 4 RGB0, two stride-2 taps per 16-B chunk): forward + BN statistics and the
    weight gradient against float64 torch, and against the one-tap-per-chunk C = 8 path."""
    N, H, W, k, s, p = case
    dtype = torch.bfloat16
    Cin, Cout = 3, 64
    x = _rand((N, Cin, H, W), dtype, 11).double()
    w = _rand((Cout, Cin, k, k), torch.float32, 12, 0.1)
    ref = F.conv2d(x, w.to(dtype).double(), stride=s, padding=p)
    OH, OW = ref.shape[2], ref.shape[3]
    outs = {}
    for cpad in (4, 8):
        xs = torch.zeros((N, H, W, cpad), dtype=dtype)
        xs[..., :Cin] = x.permute(0, 2, 3, 1).to(dtype)
        xs = xs.to(DEV)
        wd = K.weight_prep(w.to(DEV), cpad, dtype, pair_pad=p if cpad == 4 else None)
        if cpad == 4:
            assert wd.shape == (Cout, k, K.pair_taps(k, p)[0], 8)
        M = N * OH * OW
        stats = K.stats_buffer(Cout, M, DEV)
        y = K.conv_fwd(xs, wd, N, H, W, cpad, Cout, k, k, s, p, 0, 0, stats=stats)
        _close(y.permute(0, 3, 1, 2), ref, dtype, f"stem fwd cpad {cpad}")
        mean, invstd, scale, shift = (torch.empty(Cout, device=DEV) for _ in range(4))
        K.bn_finalize(stats, K.stats_tiles(M), M, Cout, torch.ones(Cout, device=DEV), torch.zeros(Cout, device=DEV),
                      mean, invstd, scale, shift, None, None, 0.1, 1e-5)
        yd = y.double().cpu().reshape(M, Cout)
        assert torch.allclose(mean.double().cpu(), yd.mean(0), atol=1e-5 * (1 + yd.mean(0).abs().max().item()))
        dy = _rand((N, Cout, OH, OW), dtype, 13).double()
        wr = w.double().requires_grad_()
        (gref,) = torch.autograd.grad(F.conv2d(x, wr, stride=s, padding=p), wr, dy)
        dw = torch.full((Cout, Cin, k, k), 0.5, dtype=torch.float32, device=DEV)
        K.conv_wgrad(xs, dy.permute(0, 2, 3, 1).contiguous().to(dtype).to(DEV), dw, N, H, W, cpad, Cin, Cout, k, k,
                     s, p, 0, 0, accumulate=True)
        _close(dw - 0.5, gref, dtype, f"stem wgrad cpad {cpad}")
        outs[cpad] = (y.float(), dw)
    # same math, different K order: the two layouts agree to fp32 summation order (+ one bf16 rounding of y)
    assert (outs[4][0] - outs[8][0]).abs().max().item() <= 1e-2 * (1 + outs[8][0].abs().max().item())
    assert (outs[4][1] - outs[8][1]).abs().max().item() <= 1e-4 * (1 + outs[8][1].abs().max().item())


def test_window_frames_u8_cpad4(K):
    """The 4-channel staging of the pair-packed stem == the first 4 channels of the 8-channel one."""
    g = torch.Generator().manual_seed(5)
    frames = torch.randint(0, 256, (5, 6, 10, 3), dtype=torch.uint8, generator=g).to(DEV)
    idx = torch.tensor([0, 4, 2, -1, 9, 3], dtype=torch.int64).to(DEV)
    for dt in (torch.bfloat16, torch.float32):
        a = K.window_frames_u8(frames, idx, dt, cpad=4)
        b = K.window_frames_u8(frames, idx, dt, cpad=8)
        assert a.shape[-1] == 4 and torch.equal(a, b[..., :4]) and not b[..., 4:].any()


@pytest.mark.parametrize("case", [(16, 28, 28, 64, 64, 3, 1, 1, 4), (8, 30, 30, 64, 256, 1, 2, 0, 0),
                                  (4, 64, 64, 3, 64, 7, 2, 3, 0), (4, 14, 14, 256, 128, 3, 2, 1, 0),
                                  (8, 20, 20, 512, 192, 1, 1, 0, 8)])
def test_conv_wgrad_split(K, case):
    """bf16 weight gradient over many pixels: split-K slabs, M = 64 / N = 64 tiles, partial N tiles
    (stem: N = 7*7*8 = 392), stride 2, TSM-shifted gather."""
    dtype = torch.bfloat16
    N, H, W, Cin, Cout, KH, s, p, T = case
    x = _rand((N, Cin, H, W), dtype, 16).double()
    fold = Cin // 8 if T else 0
    w = _rand((Cout, Cin, KH, KH), torch.float32, 17, 0.1).double().requires_grad_()
    xin = tsm_ref(x, T, fold) if T else x
    y = F.conv2d(xin, w, stride=s, padding=p)
    dy = _rand(y.shape, dtype, 18).double()
    (ref,) = torch.autograd.grad(y, w, dy)
    xs, cpad = _prep(K, x, None, dtype, T, fold)
    dys = dy.permute(0, 2, 3, 1).contiguous().to(dtype).to(DEV)
    dw = torch.zeros((Cout, Cin, KH, KH), dtype=torch.float32, device=DEV)
    K.conv_wgrad(xs, dys, dw, N, H, W, cpad, Cin, Cout, KH, KH, s, p, T, fold, accumulate=False)
    # inputs are exact bf16 values, accumulation fp32: only summation-order error
    err = (dw.double().cpu() - ref).abs().max().item()
    assert err <= 1e-4 * ref.abs().max().item() + 1e-6, f"max err {err}"


@pytest.mark.parametrize("n,off", [(133_355_074, 0), (1_000_003, 0), (1_000_003, 1), (7, 0), (4096, 3)])
def test_sumsq(K, n, off):
    """Gradient-norm reduction (vcg_sumsq: 16-B loads when aligned, a 4-B path for misaligned views, tails) against
    a float64 sum."""
    g = torch.Generator().manual_seed(n + off)
    x = torch.randn(n + off, generator=g).to(DEV)
    v = x[off:]
    out = torch.zeros(1, device=DEV)
    K.sumsq(v, out)
    ref = (v.double() ** 2).sum().item()
    assert abs(out.item() - ref) <= 1e-5 * ref


@pytest.mark.parametrize("dtype", DTYPES)
@pytest.mark.parametrize("P,C", [(4096, 256), (777, 2048), (50, 64)])
def test_bn_bwd_apply_dual(K, dtype, P, C):
    """One pass over g for bn3 and the downsample BN (vcg_bn_bwd_apply_dual) == two vcg_bn_bwd_apply calls: the same
    affine arithmetic, up to the compiler's fma contraction of the per-channel coefficients (fp32: 1e-5 relative;
    bf16: within one output rounding)."""
    g = _rand((P, C), dtype, 31).to(DEV)
    ys = [_rand((P, C), dtype, 32 + k, 3.0).to(DEV) for k in range(2)]
    prm = []
    for k in range(2):
        gen = torch.Generator().manual_seed(40 + k)
        mean, invstd, gamma, sg, sgx = (torch.randn(C, generator=gen).to(DEV) for _ in range(5))
        prm.append((mean, invstd.abs() + 0.5, gamma, sg, sgx))
    dy, dyd = K.bn_bwd_apply_dual(g, ys[0], *prm[0], ys[1], *prm[1], C)
    for out, y, (mean, invstd, gamma, sg, sgx) in ((dy, ys[0], prm[0]), (dyd, ys[1], prm[1])):
        ref = K.bn_bwd_apply(g, None, y, mean, invstd, gamma, sg, sgx, C, train_stats=True)
        o, r = out.double().cpu(), ref.double().cpu()
        tol = 1e-5 if dtype == torch.float32 else 2.0 ** -7
        assert ((o - r).abs() <= tol * r.abs() + 1e-6 * r.abs().max()).all()


@pytest.mark.parametrize("case", [(8, 56, 56, 64, 64), (1, 56, 56, 64, 64), (6, 28, 28, 64, 64), (3, 20, 20, 64, 64),
                                  (2, 13, 9, 64, 64), (4, 28, 28, 128, 128), (3, 14, 14, 256, 256),
                                  (5, 14, 14, 512, 512), (2, 14, 14, 128, 256), (3, 16, 16, 64, 192)])
def test_conv_wgrad_patch(K, case):
    """The stride-1 3x3 weight gradient on the LDS patch (wgrad3x3_patch_kernel: one workgroup per 64 x 64 channel
    block and tile range, pad 1; R rows per tile = 2 / 2 / 4 / 5 / 13 / 4 / 7 / 7 here, ragged TM, 2- and 4-step
    tiles, pitches 16 / 32 / 64, workgroups with no tile, Cin != Cout) against float64 torch."""
    dtype = torch.bfloat16
    N, H, W, C, Co = case
    x = _rand((N, C, H, W), dtype, 26).double()
    w = _rand((Co, C, 3, 3), torch.float32, 27, 0.1).double().requires_grad_()
    y = F.conv2d(x, w, stride=1, padding=1)
    dy = _rand(y.shape, dtype, 28).double()
    (ref,) = torch.autograd.grad(y, w, dy)
    xs = x.permute(0, 2, 3, 1).contiguous().to(dtype).to(DEV)
    dys = dy.permute(0, 2, 3, 1).contiguous().to(dtype).to(DEV)
    dw = torch.full((Co, C, 3, 3), 0.25, dtype=torch.float32, device=DEV)
    K.conv_wgrad(xs, dys, dw, N, H, W, C, C, Co, 3, 3, 1, 1, 0, 0, accumulate=True)
    err = (dw.double().cpu() - 0.25 - ref).abs().max().item()
    assert err <= 1e-4 * ref.abs().max().item() + 1e-6, f"max err {err}"


@pytest.mark.parametrize("dtype", DTYPES)
@pytest.mark.parametrize("tA,tB", [(0, 0), (0, 1), (1, 0), (1, 1)])
def test_gemm(K, dtype, tA, tB):
    M, N, Kd = 200, 192, 96
    A = _rand((Kd, M) if tA else (M, Kd), dtype, 9)
    B = _rand((Kd, N) if tB else (N, Kd), dtype, 10)
    bias = torch.randn(N)
    res = _rand((M, N), dtype, 11)
    Am = A.double().t() if tA else A.double()
    Bm = B.double() if tB else B.double().t()
    pre = Am @ Bm + bias.double() + res.double()
    ref = F.gelu(pre)
    aux = torch.empty((M, N), dtype=dtype, device=DEV)
    out = K.gemm(A.to(DEV), B.to(DEV), M, N, Kd, M if tA else Kd, N if tB else Kd, transA=bool(tA),
                 transB=bool(tB), bias=bias.to(DEV), act=K.ACT_GELU, residual=res.to(DEV), aux=aux)
    _close(out, ref, dtype, "gemm")
    _close(aux, pre, dtype, "gemm aux")
    # GELU backward epilogue: out = (A B^T) * gelu'(res)
    out2 = K.gemm(A.to(DEV), B.to(DEV), M, N, Kd, M if tA else Kd, N if tB else Kd, transA=bool(tA),
                  transB=bool(tB), act=K.ACT_GELU_BWD, residual=res.to(DEV))
    r = res.double()
    cdf = 0.5 * (1 + torch.erf(r / np.sqrt(2)))
    pdf = torch.exp(-0.5 * r * r) / np.sqrt(2 * np.pi)
    _close(out2, (Am @ Bm) * (cdf + r * pdf), dtype, "gemm gelu bwd")


@pytest.mark.parametrize("dtype", DTYPES)
@pytest.mark.parametrize("shape", [(64, 768, 5000, 64, 768), (200, 136, 1000, 256, 144), (768, 3072, 8192, 768, 3072)])
def test_gemm_splitk(K, dtype, shape):
    # transA = transB = 1 (dW = dY^T X of the linear layers)
    M, N, Kd, lda, ldb = shape
    A = _rand((Kd, lda), dtype, 12)
    B = _rand((Kd, ldb), dtype, 13)
    out = torch.ones((M, N), dtype=torch.float32, device=DEV)
    K.gemm_splitk(A.to(DEV), B.to(DEV), out, M, N, Kd, lda, ldb, transA=True, transB=True, accumulate=True)
    _close(out - 1, A[:, :M].double().t() @ B[:, :N].double(), dtype, "gemm splitk")


@pytest.mark.parametrize("dtype", DTYPES)
def test_gemm_batched_attention_shapes(K, dtype):
    B, L, nh, dh = 3, 40, 2, 64
    H = nh * dh
    Lp = 40
    qkv = _rand((B * L, 3 * H), dtype, 14)
    S = torch.empty((B * nh, L, Lp), dtype=dtype, device=DEV)
    q = qkv.to(DEV)
    K.gemm_batched(q, q[:, H:], S, L, Lp, dh, 3 * H, 3 * H, Lp, L * 3 * H, dh, L * 3 * H, dh, nh * L * Lp, L * Lp, B,
                   nh)
    qd = qkv.double().view(B, L, 3, nh, dh)
    ref = torch.einsum("blhd,bmhd->bhlm", qd[:, :, 0], qd[:, :, 1]).reshape(B * nh, L, L)
    _close(S, ref, dtype, "batched QK^T")


@pytest.mark.parametrize("dtype", DTYPES)
def test_bn_apply_and_bwd(K, dtype):
    N, H, W, C = 6, 5, 5, 64
    y = _rand((N, C, H, W), dtype, 15).double().requires_grad_()
    gamma = (torch.rand(C) + 0.5).double().requires_grad_()
    beta = torch.randn(C).double().requires_grad_()
    out = F.relu(F.batch_norm(y, None, None, gamma, beta, training=True, eps=1e-5))
    dout = _rand(out.shape, dtype, 16).double()
    gy, gg, gb = torch.autograd.grad(out, (y, gamma, beta), dout)
    ys = y.detach().permute(0, 2, 3, 1).contiguous().to(dtype).to(DEV)
    M = N * H * W
    # stats via finalize from a synthetic single-tile partial: compute with the conv path instead
    mean = y.detach().mean((0, 2, 3)).float().to(DEV)
    var = y.detach().var((0, 2, 3), unbiased=False)
    invstd = (1 / torch.sqrt(var + 1e-5)).float().to(DEV)
    g32, b32 = gamma.detach().float().to(DEV), beta.detach().float().to(DEV)
    scale = g32 * invstd
    shift = b32 - mean * scale
    a = K.bn_apply(ys, scale, shift, C, relu=True)
    _close(a.permute(0, 3, 1, 2), out, dtype, "bn apply")
    douts = dout.permute(0, 2, 3, 1).contiguous().to(dtype).to(DEV)
    sg = torch.empty(C, device=DEV)
    sgx = torch.empty(C, device=DEV)
    dgam = torch.zeros(C, device=DEV)
    dbet = torch.zeros(C, device=DEV)
    K.bn_bwd_reduce(douts, a, ys, mean, invstd, C, sg, sgx, dgam, dbet)
    dy = K.bn_bwd_apply(douts, a, ys, mean, invstd, g32, sg, sgx, C, train_stats=True)
    _close(dy.permute(0, 3, 1, 2), gy, dtype, "bn bwd dx")
    _close(dgam, gg, dtype, "bn dgamma")
    _close(dbet, gb, dtype, "bn dbeta")
    # the mask recomputed from y (mode 3) and the forward's mask bits (mode 2) give the same bits
    a2, bits = K.bn_apply(ys, scale, shift, C, relu=True, bits=True)
    assert torch.equal(a2, a)
    ref_bits = (a.reshape(-1, 16 // a.element_size()) > 0).to(torch.int32)
    weights = 2 ** torch.arange(ref_bits.shape[1], device=DEV, dtype=torch.int32)
    assert torch.equal(bits.to(torch.int32), (ref_bits * weights).sum(1))
    for kw in ({"mscale": scale, "mshift": shift}, {"mbits": bits}):
        sg2, sgx2 = torch.empty(C, device=DEV), torch.empty(C, device=DEV)
        K.bn_bwd_reduce(douts, None, ys, mean, invstd, C, sg2, sgx2, **kw)
        dy2 = K.bn_bwd_apply(douts, None, ys, mean, invstd, g32, sg2, sgx2, C, train_stats=True, **kw)
        assert torch.equal(sg2, sg) and torch.equal(sgx2, sgx), kw.keys()
        assert torch.equal(dy2, dy), kw.keys()


def test_tsm_unshift_masked_residual(K):
    """dx = unshift(dshift) + other * mask(bits) == unshift(dshift) + (other where out > 0)."""
    dtype = torch.bfloat16
    NT, T, HW, C, fold = 16, 8, 9, 64, 8
    dsh = _rand((NT, HW, C), dtype, 41).to(DEV)
    oth = _rand((NT, HW, C), dtype, 42).to(DEV)
    y = _rand((NT, HW, C), dtype, 43).to(DEV)
    one = torch.ones(C, device=DEV)
    zero = torch.zeros(C, device=DEV)
    a, bits = K.bn_apply(y, one, zero, C, relu=True, bits=True)
    dx = K.tsm_unshift_add(dsh, oth, NT, T, HW, C, fold, other_bits=bits)
    ref = K.tsm_unshift_add(dsh, torch.where(a > 0, oth, torch.zeros_like(oth)), NT, T, HW, C, fold)
    assert torch.equal(dx, ref)


@pytest.mark.parametrize("dtype", DTYPES)
def test_maxpool(K, dtype):
    N, C, H, W = 3, 64, 11, 12
    x = F.relu(_rand((N, C, H, W), dtype, 17)).double().requires_grad_()  # relu -> many ties at 0
    y = F.max_pool2d(x, 3, 2, 1)
    dy = _rand(y.shape, dtype, 18).double()
    (gx,) = torch.autograd.grad(y, x, dy)
    xs = x.detach().permute(0, 2, 3, 1).contiguous().to(dtype).to(DEV)
    ys, idx = K.maxpool_fwd(xs, N, H, W, C)
    _close(ys.permute(0, 3, 1, 2), y, dtype, "maxpool fwd")
    dys = dy.permute(0, 2, 3, 1).contiguous().to(dtype).to(DEV)
    dx = K.maxpool_bwd(dys, idx, N, H, W, C)
    _close(dx.permute(0, 3, 1, 2), gx, dtype, "maxpool bwd")


@pytest.mark.parametrize("dtype", DTYPES)
def test_tsm_shift_bitexact(K, dtype):
    x = _rand((2 * 8, 64, 7, 7), dtype, 19)
    ref = tsm_ref(x, 8, 64 // 8)
    y = K.tsm_shift(x.to(DEV), 8, 8, direction=0)
    assert torch.equal(y.cpu(), ref)
    # adjoint: <shift(x), g> == <x, shift^T(g)>
    g = _rand(x.shape, torch.float32, 20)
    gt = K.tsm_shift(g.to(DEV), 8, 8, direction=1).cpu()
    xr = x.double()
    assert abs((tsm_ref(xr, 8, 8) * g.double()).sum() - (xr * gt.double()).sum()) < 1e-6 * x.numel()


def test_avgpool(K):
    x = torch.randn(4, 49, 256)
    y = K.avgpool_fwd(x.to(DEV), 4, 49, 256)
    _close(y, x.double().mean(1), torch.float32, "avgpool")


@pytest.mark.parametrize("N,HW,C", [(64, 49, 2048), (3, 5, 8), (2, 9, 24)])
def test_avgpool_bf16(K, N, HW, C):
    """The trunk's global average pool and its backward in bf16 (8 channels per thread) vs float64."""
    x = _rand((N, HW, C), torch.bfloat16, 51)
    y = K.avgpool_fwd(x.to(DEV), N, HW, C)
    ref = x.double().mean(1)
    assert (y.double().cpu() - ref).abs().max().item() <= 1e-5 * (ref.abs().max().item() + 1.0)
    dy = torch.randn(N, C)
    dx = K.avgpool_bwd(dy.to(DEV), N, HW, C, torch.bfloat16)
    assert torch.equal(dx.cpu(), (dy / HW).to(torch.bfloat16)[:, None, :].expand(N, HW, C))


def test_window_frames_u8_bitexact(K):
    """Frame ingest: u8 frames gathered by the window frame table (data/clip_windows.py) and
    normalised like ToTensor + Normalize in fp32 — bit-exact in fp32, one rounding in bf16."""
    from data import clip_windows as cw
    g = torch.Generator().manual_seed(31)
    F_, H, W, T = 40, 12, 10, 16
    frames = torch.randint(0, 256, (F_, H, W, 3), generator=g, dtype=torch.uint8)
    win = cw.clip_windows(F_, T)
    idx = torch.from_numpy(cw.frame_index_table(win, F_))
    mean = torch.tensor(K.IMAGENET_MEAN, dtype=torch.float32)
    std = torch.tensor(K.IMAGENET_STD, dtype=torch.float32)
    ref = (frames[idx.reshape(-1)].float() / 255.0 - mean) / std          # [n,H,W,3] fp32
    for dt in (torch.float32, torch.bfloat16):
        y = K.window_frames_u8(frames.to(DEV), idx.to(DEV), dt).cpu()
        assert y.shape == (idx.numel(), H, W, 8)
        assert torch.equal(y[..., 3:], torch.zeros_like(y[..., 3:]))
        assert torch.equal(y[..., :3], ref.to(dt)), dt


@pytest.mark.parametrize("dtype", DTYPES)
@pytest.mark.parametrize("shape", [(2304, 768), (70, 129), (1, 64)])
def test_transpose(K, dtype, shape):
    x = _rand(shape, dtype, 21)
    y = K.transpose(x.to(DEV))
    assert torch.equal(y.cpu(), x.t().contiguous()), "transpose must be an exact copy"


def test_transpose_multi(K):
    """The batched bf16 transpose (BERT's W^T cache) against torch, several shapes in one launch (ragged tiles)."""
    shapes = [(2304, 768), (768, 3072), (72, 200), (8, 8), (64, 128)]
    xs = [_rand(s, torch.bfloat16, 30 + i).to(DEV) for i, s in enumerate(shapes)]
    outs = [torch.empty((s[1], s[0]), dtype=torch.bfloat16, device=DEV) for s in shapes]
    desc, tiles = [], 0
    for x, o in zip(xs, outs):
        r, c = x.shape
        desc.append([x.data_ptr(), o.data_ptr(), r, c, tiles])
        tiles += ((r + 63) // 64) * ((c + 63) // 64)
    K.transpose_multi(torch.tensor(desc, dtype=torch.int64).to(DEV), len(desc), tiles)
    for x, o in zip(xs, outs):
        assert torch.equal(o, x.t().contiguous())


# (N, H, W, C = dgrad output channels, Cout, k, stride, pad, T) of the fused trunk-backward dgrad
DGRAD_BWD_CASES = [
    (16, 65, 71, 128, 64, 3, 1, 1, 4),  # >= 64 Ki rows, 128 columns
    (16, 64, 70, 256, 64, 1, 1, 0, 8),  # same, dense 1x1
    (8, 9, 9, 64, 64, 3, 1, 1, 4),     # conv2 3x3
    (8, 10, 10, 64, 128, 3, 2, 1, 4),  # conv2 3x3 / 2 (block 0 of a stage): four sub-pixel class GEMMs
    (16, 28, 28, 128, 128, 3, 2, 1, 4),  # same, several tiles per class
    (8, 7, 7, 64, 256, 1, 1, 0, 4),    # conv3 / conv1 1x1 (dense)
    (8, 6, 6, 128, 64, 1, 1, 0, 8),    # wider C: BN = 128 tiles
    (8, 7, 9, 256, 128, 1, 1, 0, 4),   # 1x1, K = 128 (streaming kernel, 3-deep ring), M = 504: a ragged last tile
    (4, 14, 14, 512, 64, 1, 1, 0, 4),  # 1x1, K = 64, 8 column tiles (streaming kernel, 4-deep ring), fold 64
]


@pytest.mark.parametrize("case", DGRAD_BWD_CASES)
@pytest.mark.parametrize("mode", ["affine", "tsm_bits_two", "tsm_plain", "tsm_strided_res"])
def test_conv_dgrad_bwd(K, case, mode):
    """Fused dgrad epilogue == the unfused ops (dgrad, TSM combine, masks) bit for bit; its BN sums == a
    float64 reduction of the same g."""
    dtype = torch.bfloat16
    N, H, W, C, Cout, k, s, p, T = case
    OH, OW = K.conv_out_hw(H, W, k, k, s, p)
    dy = _rand((N, OH, OW, Cout), dtype, 61).to(DEV)
    w = _rand((Cout, C, k, k), torch.float32, 62, 0.1).to(DEV)
    wt = K.weight_prep(w, C, dtype, transposed=True)
    y = _rand((N, H, W, C), dtype, 63).to(DEV)
    y2 = _rand((N, H, W, C), dtype, 64).to(DEV)
    res = _rand((N, H, W, C), dtype, 65).to(DEV)
    g0 = torch.Generator().manual_seed(66)
    mean = (torch.randn(C, generator=g0) * 0.1).to(DEV)
    inv = (torch.rand(C, generator=g0) + 0.5).to(DEV)
    # dyadic mask parameters: y * msc + msh is exact in f32, so torch's unfused test == the kernel's fma
    msc = (torch.tensor([0.5, 1.0, 2.0, -0.5, -1.0, -2.0])[torch.randint(0, 6, (C,), generator=g0)]).to(DEV)
    msh = (torch.randint(-16, 17, (C,), generator=g0).float() / 64).to(DEV)
    mean2 = (torch.randn(C, generator=g0) * 0.1).to(DEV)
    inv2 = (torch.rand(C, generator=g0) + 0.5).to(DEV)
    dx = K.conv_dgrad(dy, wt, N, H, W, C, Cout, k, k, s, p)
    sums = torch.zeros((2, C), device=DEV)
    sgx2 = torch.zeros(C, device=DEV)
    dgam, dbet = torch.full((C,), 0.5, device=DEV), torch.full((C,), 0.25, device=DEV)
    dgam2, dbet2 = torch.full((C,), 0.5, device=DEV), torch.full((C,), 0.25, device=DEV)
    if mode == "affine":
        g = K.conv_dgrad_bwd(dy, wt, N, H, W, C, Cout, k, k, s, p, y=y, mean=mean, invstd=inv, mscale=msc,
                             mshift=msh, sums=sums, dgamma=dgam, dbeta=dbet)
        keep = y.float() * msc + msh > 0
        ref = torch.where(keep, dx, torch.zeros_like(dx))
    else:
        fold = C // 8
        _, bits = K.bn_apply(y2, torch.ones(C, device=DEV), torch.zeros(C, device=DEV), C, relu=True, bits=True)
        comb = K.tsm_unshift_add(dx, res, N, T, H * W, C, fold)
        if mode == "tsm_plain":
            g = K.conv_dgrad_bwd(dy, wt, N, H, W, C, Cout, k, k, s, p, tsm_T=T, tsm_fold=fold, res=res)
            ref = comb
        elif mode == "tsm_strided_res":
            # compact residual of a 1x1 / stride-2 downsample: only even (h, w) rows receive it
            rc = _rand((N, (H + 1) // 2, (W + 1) // 2, C), dtype, 67).to(DEV)
            full = torch.zeros_like(res)
            full[:, ::2, ::2, :] = rc
            g = K.conv_dgrad_bwd(dy, wt, N, H, W, C, Cout, k, k, s, p, tsm_T=T, tsm_fold=fold, res=rc, res_stride=2)
            ref = K.tsm_unshift_add(dx, full, N, T, H * W, C, fold)
        else:
            g = K.conv_dgrad_bwd(dy, wt, N, H, W, C, Cout, k, k, s, p, tsm_T=T, tsm_fold=fold, res=res, bits=bits,
                                 y=y, mean=mean, invstd=inv, y2=y2, mean2=mean2, invstd2=inv2, sums=sums,
                                 sum_gx2=sgx2, dgamma=dgam, dbeta=dbet, dgamma2=dgam2, dbeta2=dbet2)
            ref = torch.where(y2 > 0, comb, torch.zeros_like(comb))
    assert g is not None, "the fused bf16 engine must take this shape"
    assert torch.equal(g, ref), f"g differs: max {(g.float() - ref.float()).abs().max().item():.3e}"
    if mode in ("tsm_plain", "tsm_strided_res"):
        return
    gd = g.double().reshape(-1, C)
    sg = gd.sum(0)
    sx = (gd * (y.double().reshape(-1, C) - mean.double()) * inv.double()).sum(0)
    tol = lambda r: 1e-4 * (r.abs().max().item() + 1.0)  # noqa: E731
    assert (sums[0].double() - sg).abs().max().item() <= tol(sg)
    assert (sums[1].double() - sx).abs().max().item() <= tol(sx)
    assert (dbet.double() - 0.25 - sg).abs().max().item() <= tol(sg)
    assert (dgam.double() - 0.5 - sx).abs().max().item() <= tol(sx)
    if mode == "tsm_bits_two":
        sx2 = (gd * (y2.double().reshape(-1, C) - mean2.double()) * inv2.double()).sum(0)
        assert (sgx2.double() - sx2).abs().max().item() <= tol(sx2)
        assert (dgam2.double() - 0.5 - sx2).abs().max().item() <= tol(sx2)
        assert (dbet2.double() - 0.25 - sg).abs().max().item() <= tol(sg)


# the trunk's conv1 input gradients that the streaming EPI_BWD kernel takes (layers 1-3 at 16 frames; K = 256: layer 3,
# one A tile per ring slot and the weights in registers): (N, H, W, C, Cout, T, res_stride)
STREAM_CASES = [(16, 56, 56, 256, 64, 8, 1), (16, 28, 28, 512, 128, 8, 1), (16, 56, 56, 256, 128, 8, 2),
                (16, 14, 14, 1024, 256, 8, 1), (16, 28, 28, 512, 256, 8, 2), (5, 14, 14, 1024, 256, 5, 1)]


@pytest.mark.parametrize("case", STREAM_CASES)
@pytest.mark.parametrize("ops_", ["y", "y2", "bits"])
def test_conv_dgrad_bwd_stream_vs_persistent(K, case, ops_, monkeypatch):
    """The streaming fused 1x1 dgrad (EPI_BWD_STREAM: A rows and residual / y / mask operands DMA'd into an LDS ring
    tiles ahead) against the persistent engine's EPI_BWD (VCG_BWD_STREAM=0) at the trunk's shapes: g bit for bit,
    the BN sums to float rounding (different tilings sum in different orders). ops_: the epilogue operands (y + mask
    bits, + the downsample's y2, or the mask bits alone: the trunk's blocks whose previous y3 is not stored)."""
    N, H, W, C, Cout, T, rs = case
    y2 = ops_ == "y2"
    dtype = torch.bfloat16
    fold = C // 8
    dy = _rand((N, H, W, Cout), dtype, 71).to(DEV)
    wt = K.weight_prep(_rand((Cout, C, 1, 1), torch.float32, 72, 0.1).to(DEV), C, dtype, transposed=True)
    y = _rand((N, H, W, C), dtype, 73).to(DEV)
    y2t = _rand((N, H, W, C), dtype, 74).to(DEV) if y2 else None
    res = _rand((N, (H + 1) // 2, (W + 1) // 2, C) if rs == 2 else (N, H, W, C), dtype, 75).to(DEV)
    _, bits = K.bn_apply(_rand((N, H, W, C), dtype, 76).to(DEV), torch.ones(C, device=DEV),
                         torch.zeros(C, device=DEV), C, relu=True, bits=True)
    g0 = torch.Generator().manual_seed(77)
    mean, inv = (torch.randn(C, generator=g0) * 0.1).to(DEV), (torch.rand(C, generator=g0) + 0.5).to(DEV)
    mean2, inv2 = (torch.randn(C, generator=g0) * 0.1).to(DEV), (torch.rand(C, generator=g0) + 0.5).to(DEV)
    outs = []
    for flag in ("1", "64", "0"):  # streaming (64 x 128 tiles where they apply), streaming 64 x 64, persistent
        monkeypatch.setenv("VCG_BWD_STREAM", flag)
        sums, sgx2 = torch.zeros((2, C), device=DEV), torch.zeros(C, device=DEV)
        kw = dict(y2=y2t, mean2=mean2, invstd2=inv2, sum_gx2=sgx2) if y2 else {}
        g = K.conv_dgrad_bwd(dy, wt, N, H, W, C, Cout, 1, 1, 1, 0, tsm_T=T, tsm_fold=fold, res=res, res_stride=rs,
                             bits=bits, y=None if ops_ == "bits" else y, mean=mean, invstd=inv, sums=sums, **kw)
        assert g is not None
        torch.cuda.synchronize()
        outs.append((g.clone(), sums.clone(), sgx2.clone()))
    gb, sb, xb = outs[-1]
    for ga, sa, xa in outs[:-1]:
        assert torch.equal(ga, gb), f"g differs: max {(ga.float() - gb.float()).abs().max().item():.3e}"
        for a, b in ((sa, sb), (xa, xb)):
            assert (a.double() - b.double()).abs().max().item() <= 1e-4 * (b.abs().max().item() + 1.0)


@pytest.mark.parametrize("dtype", DTYPES)
@pytest.mark.parametrize("H,rows", [(768, 37), (200, 37), (768, 2085)])
def test_layernorm_fwd_bwd(K, dtype, H, rows):
    """LN(x + res) forward / backward (row-wise wave kernels at H = 768, block kernels at H = 200) against
    torch autograd in float64; the fused bias gradient = column sums of dx. 2085 rows: every wave of the row-wise
    backward walks several rows (the next row's operands prefetched under this row's arithmetic)."""
    x = _rand((rows, H), dtype, 71)
    r = _rand((rows, H), dtype, 72)
    g0 = torch.Generator().manual_seed(73)
    gamma = torch.rand(H, generator=g0) + 0.5
    beta = torch.randn(H, generator=g0) * 0.1
    dout = _rand((rows, H), dtype, 74)
    xd = x.double().requires_grad_()
    rd = r.double().requires_grad_()
    gd = gamma.double().requires_grad_()
    bd = beta.double().requires_grad_()
    y = F.layer_norm(xd + rd, (H,), gd, bd, eps=1e-12)
    dx_ref, dr_ref, dg_ref, db_ref = torch.autograd.grad(y, (xd, rd, gd, bd), dout.double())
    out, mean, rstd = K.ln_fwd(x.to(DEV), r.to(DEV), gamma.to(DEV), beta.to(DEV), rows, H, 1e-12)
    _close(out, y, dtype, "ln fwd")
    gg = torch.zeros(H, device=DEV)
    gb = torch.zeros(H, device=DEV)
    gbias = torch.full((H,), 0.5, device=DEV)
    dx, dres = K.ln_bwd(dout.to(DEV), x.to(DEV), r.to(DEV), gamma.to(DEV), mean, rstd, gg, gb, rows, H,
                        bias_grad=gbias)
    _close(dx, dx_ref, dtype, "ln bwd dx")
    _close(dres, dr_ref, dtype, "ln bwd dres")
    _close(gg, dg_ref, dtype, "ln dgamma")
    _close(gb, db_ref, dtype, "ln dbeta")
    _close(gbias - 0.5, dx.double().sum(0), torch.float32, "ln fused bias grad")
    cs = torch.full((H,), 0.25, device=DEV)
    K.colsum(dx, H, rows, H, cs)
    _close(cs - 0.25, dx.double().sum(0), torch.float32, "colsum")


@pytest.mark.parametrize("H,rows", [(768, 37), (768, 2085), (512, 300)])
def test_layernorm_bwd_fp32_gradient_stream(K, H, rows):
    """LN backward with bf16 x / res and an fp32 incoming gradient (VCG_GRAD_F32, BERT's fp32 residual-gradient
    stream): dres comes back fp32 and dx bf16; both closer to float64 autograd than the all-bf16 call on the
    bf16-rounded gradient (dres to fp32 rounding of the same arithmetic), dgamma / dbeta likewise."""
    x = _rand((rows, H), torch.bfloat16, 171)
    r = _rand((rows, H), torch.bfloat16, 172)
    g0 = torch.Generator().manual_seed(173)
    gamma = torch.rand(H, generator=g0) + 0.5
    beta = torch.randn(H, generator=g0) * 0.1
    dout = torch.randn(rows, H, generator=g0)  # fp32
    xd, rd = x.double().requires_grad_(), r.double().requires_grad_()
    y = F.layer_norm(xd + rd, (H,), gamma.double(), beta.double(), eps=1e-12)
    dx_ref, dr_ref = torch.autograd.grad(y, (xd, rd), dout.double())
    _, mean, rstd = K.ln_fwd(x.to(DEV), r.to(DEV), gamma.to(DEV), beta.to(DEV), rows, H, 1e-12)
    res = {}
    for tag, d in (("f32", dout.to(DEV)), ("bf16", dout.to(torch.bfloat16).to(DEV))):
        gg, gb = torch.zeros(H, device=DEV), torch.zeros(H, device=DEV)
        dx, dres = K.ln_bwd(d, x.to(DEV), r.to(DEV), gamma.to(DEV), mean, rstd, gg, gb, rows, H)
        res[tag] = (dx, dres)
    dx32, dres32 = res["f32"]
    assert dx32.dtype == torch.bfloat16 and dres32.dtype == torch.float32
    e = {t: ((res[t][1].double().cpu() - dr_ref).norm() / dr_ref.norm()).item() for t in res}
    assert e["f32"] < 1e-5, e  # the fp32 stream: fp32 rounding only
    assert e["f32"] < 0.1 * e["bf16"], e
    _close(dx32, dx_ref, torch.bfloat16, "ln bwd dx (fp32 dout)")


def test_maxpool_bwd_bn(K):
    """maxpool backward fused with the stem BN mask + reduction == maxpool_bwd, masked; sums in float64."""
    dtype = torch.bfloat16
    N, C, H, W = 3, 64, 13, 12
    x = F.relu(_rand((N, H, W, C), dtype, 81)).to(DEV)
    ys, idx = K.maxpool_fwd(x, N, H, W, C)
    dys = _rand(ys.shape, dtype, 82).to(DEV)
    y = _rand((N, H, W, C), dtype, 83).to(DEV)
    g0 = torch.Generator().manual_seed(84)
    msc = (torch.tensor([0.5, 1.0, 2.0, -0.5, -1.0, -2.0])[torch.randint(0, 6, (C,), generator=g0)]).to(DEV)
    msh = (torch.randint(-16, 17, (C,), generator=g0).float() / 64).to(DEV)
    mean = (torch.randn(C, generator=g0) * 0.1).to(DEV)
    inv = (torch.rand(C, generator=g0) + 0.5).to(DEV)
    sums = torch.zeros((2, C), device=DEV)
    dg, db = torch.full((C,), 0.5, device=DEV), torch.full((C,), 0.25, device=DEV)
    g = K.maxpool_bwd_bn(dys, idx, N, H, W, C, y, mean, inv, msc, msh, sums, dg, db)
    dx = K.maxpool_bwd(dys, idx, N, H, W, C)
    ref = torch.where(y.float() * msc + msh > 0, dx, torch.zeros_like(dx))
    assert torch.equal(g, ref)
    gd = g.double().reshape(-1, C)
    sg = gd.sum(0)
    sx = (gd * (y.double().reshape(-1, C) - mean.double()) * inv.double()).sum(0)
    assert (sums[0].double() - sg).abs().max().item() <= 1e-4 * (sg.abs().max().item() + 1)
    assert (sums[1].double() - sx).abs().max().item() <= 1e-4 * (sx.abs().max().item() + 1)
    assert (db.double() - 0.25 - sg).abs().max().item() <= 1e-4 * (sg.abs().max().item() + 1)
    assert (dg.double() - 0.5 - sx).abs().max().item() <= 1e-4 * (sx.abs().max().item() + 1)


@pytest.mark.parametrize("dtype", DTYPES)
@pytest.mark.parametrize("train", [True, False])
@pytest.mark.parametrize("hw", [(13, 12), (14, 12), (16, 10), (112, 112)])
def test_fused_stem_bn_relu_maxpool(K, dtype, train, hw):
    """The fused stem passes == the unfused ops, bit for bit: bn_relu_maxpool == bn_apply(relu) + maxpool_fwd
    (values and argmax); maxpool_bwd_bn(store_g=False) + maxpool_bwd_bn_apply == maxpool_bwd_bn + bn_bwd_apply.
    Even H and W take the 2x2-block backward kernel, odd ones the per-pixel kernel: both == maxpool_bwd masked."""
    N, C = 3, 64
    H, W = hw
    y = _rand((N, H, W, C), dtype, 85).to(DEV)
    g0 = torch.Generator().manual_seed(86)
    sc = (torch.rand(C, generator=g0) * 2 - 0.5).to(DEV)   # some negative scales: no monotonicity shortcut
    sh = (torch.randn(C, generator=g0) * 0.3).to(DEV)
    a = K.bn_apply(y, sc, sh, C, relu=True)
    mp_ref, idx_ref = K.maxpool_fwd(a, N, H, W, C)
    mp, idx = K.bn_relu_maxpool(y, sc, sh, N, H, W, C)
    assert torch.equal(mp, mp_ref) and torch.equal(idx, idx_ref)
    dys = _rand(mp.shape, dtype, 87).to(DEV)
    mean = (torch.randn(C, generator=g0) * 0.1).to(DEV)
    inv = (torch.rand(C, generator=g0) + 0.5).to(DEV)
    gamma = (torch.rand(C, generator=g0) + 0.5).to(DEV)
    s_ref, s_new = torch.zeros((2, C), device=DEV), torch.zeros((2, C), device=DEV)
    g = K.maxpool_bwd_bn(dys, idx, N, H, W, C, y, mean, inv, sc, sh, s_ref)
    plain = K.maxpool_bwd(dys, idx, N, H, W, C)
    assert torch.equal(g, torch.where(y.float() * sc + sh > 0, plain, torch.zeros_like(plain)))
    dx_ref = K.bn_bwd_apply(g, None, y, mean, inv, gamma, s_ref[0], s_ref[1], C, train_stats=train)
    assert K.maxpool_bwd_bn(dys, idx, N, H, W, C, y, mean, inv, sc, sh, s_new, store_g=False) is None
    assert torch.equal(s_new, s_ref)
    dx = K.maxpool_bwd_bn_apply(dys, idx, N, H, W, C, y, mean, inv, sc, sh, gamma, s_new, N * H * W, train)
    assert torch.equal(dx, dx_ref)


@pytest.mark.parametrize("train", [True, False])
@pytest.mark.parametrize("shape", [(2, 32, 32), (3, 24, 40), (2, 56, 56), (1, 112, 112)])
def test_stem_bwd_fused(K, train, shape):
    """The one-pass stem backward (max-pool + BN + ReLU backward contracted with the frames into the 7x7 / 2 conv's
    weight gradient, dy0 only in LDS) == maxpool_bwd_bn_apply + conv_wgrad (the pair-packed stem engine): the same
    dy0 (bit-exact arithmetic), products summed in another order, so 1e-4 relative; accumulate adds."""
    N, H1, W1 = shape
    C = 64
    g0 = torch.Generator().manual_seed(92)
    y = _rand((N, H1, W1, C), torch.bfloat16, 93).to(DEV)
    sc = (torch.rand(C, generator=g0) * 2 - 0.5).to(DEV)
    sh = (torch.randn(C, generator=g0) * 0.3).to(DEV)
    mp, idx = K.bn_relu_maxpool(y, sc, sh, N, H1, W1, C)
    dys = _rand(mp.shape, torch.bfloat16, 94).to(DEV)
    mean = (torch.randn(C, generator=g0) * 0.1).to(DEV)
    inv = (torch.rand(C, generator=g0) + 0.5).to(DEV)
    gamma = (torch.rand(C, generator=g0) + 0.5).to(DEV)
    sums = torch.zeros((2, C), device=DEV)
    K.maxpool_bwd_bn(dys, idx, N, H1, W1, C, y, mean, inv, sc, sh, sums, store_g=False)
    xs = torch.zeros((N, 2 * H1, 2 * W1, 4), dtype=torch.bfloat16)
    xs[..., :3] = _rand((N, 2 * H1, 2 * W1, 3), torch.bfloat16, 95)
    xs = xs.to(DEV)
    dy0 = K.maxpool_bwd_bn_apply(dys, idx, N, H1, W1, C, y, mean, inv, sc, sh, gamma, sums, N * H1 * W1, train)
    ref = torch.zeros((C, 3, 7, 7), device=DEV)
    K.conv_wgrad(xs, dy0, ref, N, 2 * H1, 2 * W1, 4, 3, C, 7, 7, 2, 3)
    out = torch.full((C, 3, 7, 7), 0.5, device=DEV)
    K.stem_bwd_fused(dys, idx, y, xs, N, H1, W1, mean, inv, sc, sh, gamma, sums, N * H1 * W1, train, out)
    torch.cuda.synchronize()
    err = (out - 0.5 - ref).abs().max().item()
    assert err <= 1e-4 * (ref.abs().max().item() + 1e-6), err
    # exact-arithmetic cross-check of the reference path itself: dy0 (as stored) contracted in fp64
    ref64 = torch.nn.grad.conv2d_weight(xs[..., :3].permute(0, 3, 1, 2).double().cpu(), (C, 3, 7, 7),
                                        dy0.permute(0, 3, 1, 2).double().cpu(), stride=2, padding=3)
    assert (out.double().cpu() - 0.5 - ref64).abs().max().item() <= 1e-4 * ref64.abs().max().item()
    out2 = torch.zeros_like(out)
    K.stem_bwd_fused(dys, idx, y, xs, N, H1, W1, mean, inv, sc, sh, gamma, sums, N * H1 * W1, train, out2)
    assert torch.equal(out2, out - 0.5) or (out2 - (out - 0.5)).abs().max().item() <= 1e-6 * ref.abs().max().item()


def test_weight_prep_multi(K):
    """One vcg_weight_prep_multi launch (LDS-tiled transposes) == vcg_weight_prep per weight and layout, bit for
    bit: 1x1 / 3x3 / 7x7 shapes, Cout and Cin*KH*KW not multiples of 64, channel padding, the pair-packed stem."""
    shapes = [(64, 64, 3, 3, 64, 0), (64, 64, 3, 3, 64, 1), (256, 64, 1, 1, 64, 0), (256, 64, 1, 1, 64, 1),
              (512, 512, 3, 3, 512, 0), (512, 512, 3, 3, 512, 1), (2048, 1024, 1, 1, 1024, 1), (70, 37, 3, 3, 40, 0),
              (70, 37, 3, 3, 37, 1), (64, 3, 7, 7, 8, 0), (64, 3, 7, 7, 4, 5), (24, 600, 3, 3, 600, 0)]
    g = torch.Generator().manual_seed(91)
    desc, outs, refs = [], [], []
    for Cout, Cin, KH, KW, cpad, mode in shapes:
        w = (torch.randn((Cout, Cin, KH, KW), generator=g) * 0.1).to(DEV)
        if mode >= 2:
            ref = K.weight_prep(w, cpad, torch.bfloat16, pair_pad=mode - 2)
        else:
            ref = K.weight_prep(w, cpad, torch.bfloat16, transposed=bool(mode))
        out = torch.full_like(ref, float("nan"))
        desc.append([w.data_ptr(), out.data_ptr(), Cout, Cin, KH, KW, cpad, mode])
        outs.append((w, out))
        refs.append(ref)
    K.weight_prep_multi(torch.tensor(desc, dtype=torch.int64).to(DEV), len(desc))
    torch.cuda.synchronize()
    for (w, out), ref, sh in zip(outs, refs, shapes):
        assert torch.equal(out.view(torch.int16), ref.view(torch.int16)), sh


@pytest.mark.parametrize("dtype", DTYPES)
@pytest.mark.parametrize("hw,degen", [((13, 12), False), ((16, 10), False), ((112, 112), False), ((16, 10), True),
                                      ((112, 112), True)])
def test_maxpool_bwd_bn_sums_pooled(K, dtype, hw, degen):
    """The stem BN-backward sums from the pooled activation (a window's gradient reaches its argmax pixel, whose
    activation is mp) == the per-pixel pass over y, up to rounding: the per-pixel pass sums g rounded to dtype per
    pixel (after adding the <= 4 windows' dy), and for g*xhat recovers nothing (y is read), while the pooled pass
    recovers y as (mp - shift) / scale, exact up to mp's rounding to dtype (bf16: 2^-9 relative per term).
    degen: channels with a zero BN scale (either sign of the shift) and a tiny one, where mp says nothing about y:
    the kernel reads y at the argmax pixel for them (finite sums equal to the per-pixel pass)."""
    N, C = 3, 64
    H, W = hw
    y = _rand((N, H, W, C), dtype, 88).to(DEV)
    g0 = torch.Generator().manual_seed(89)
    sc = (torch.rand(C, generator=g0) * 2 - 0.5).to(DEV)
    sc = torch.where(sc.abs() < 0.05, torch.full_like(sc, 0.05), sc)
    sh = (torch.randn(C, generator=g0) * 0.3).to(DEV)
    if degen:
        sc[3], sh[3] = 0.0, 0.4
        sc[9], sh[9] = 0.0, -0.2
        sc[17], sh[17] = 0.0, 0.0
        sc[40], sh[40] = 1e-4, 0.5
    mp, idx = K.bn_relu_maxpool(y, sc, sh, N, H, W, C)
    dys = _rand(mp.shape, dtype, 90).to(DEV)
    mean = (torch.randn(C, generator=g0) * 0.1).to(DEV)
    inv = (torch.rand(C, generator=g0) + 0.5).to(DEV)
    s_ref, s_new = torch.zeros((2, C), device=DEV), torch.zeros((2, C), device=DEV)
    dg, db = torch.full((C,), 0.5, device=DEV), torch.full((C,), 0.25, device=DEV)
    K.maxpool_bwd_bn(dys, idx, N, H, W, C, y, mean, inv, sc, sh, s_ref, store_g=False)
    K.maxpool_bwd_bn_sums_pooled(dys, mp, idx, y, N, H, W, C, mean, inv, sc, sh, s_new, dg, db)
    torch.cuda.synchronize()
    assert torch.isfinite(s_new).all()
    tol = 1e-5 if dtype == torch.float32 else 4e-3
    for k in range(2):
        scale = s_ref[k].abs().max().item() + 1
        assert (s_new[k] - s_ref[k]).abs().max().item() <= tol * scale, k
    assert torch.allclose(db - 0.25, s_new[0], atol=1e-6) and torch.allclose(dg - 0.5, s_new[1], atol=1e-6)


def test_attention_softmax_dropout(K):
    """Masked softmax + dropout: P matches torch softmax over the valid keys; Pd = P / (1 - p) on kept
    entries and 0 on dropped ones (drop rate ~ p); the backward regenerates the same mask."""
    B, nh, L, Lp, p = 2, 3, 40, 40, 0.1
    Z = B * nh
    S = torch.randn(Z, L, Lp).to(DEV)
    mask = torch.ones(B, L, dtype=torch.int64)
    mask[1, 30:] = 0
    mask = mask.to(DEV)
    Pm, Pd = torch.empty_like(S), torch.empty_like(S)
    K.attn_softmax_fwd(S, mask, Pm, Pd, B, nh, L, Lp, 0.125, p, seed=1234)
    add = torch.where(mask.bool(), 0.0, float("-inf")).repeat_interleave(nh, 0)[:, None, :]
    ref = torch.softmax(S.double() * 0.125 + add.double(), -1)
    assert (Pm.double() - ref).abs().max().item() < 1e-5
    kept = Pd != 0
    valid = ref > 0
    rate = 1 - kept[valid].float().mean().item()
    assert abs(rate - p) < 0.02, f"drop rate {rate:.3f}"
    assert torch.allclose(Pd[kept], Pm[kept] / (1 - p), rtol=1e-6, atol=0)
    dS = torch.empty_like(S)
    K.attn_softmax_bwd(torch.ones_like(S), Pm, dS, Z, L, Lp, 0.125, p, seed=1234)
    dp = kept.double() / (1 - p)
    dot = (dp * Pm.double()).sum(-1, keepdim=True)
    assert (dS.double() - 0.125 * Pm.double() * (dp - dot)).abs().max().item() < 1e-5


@pytest.mark.parametrize("case", [(16, 65, 71, 128, 64, 3, 1, 1), (16, 64, 70, 256, 64, 1, 1, 0),
                                  (8, 130, 66, 128, 64, 3, 2, 1)])
def test_conv_dgrad_big(K, case):
    """Input gradients with >= 64 Ki rows against torch in float64."""
    dtype = torch.bfloat16
    N, H, W, Cin, Cout, KH, s, p = case
    x = torch.zeros((N, Cin, H, W), dtype=torch.float64, requires_grad=True)
    w = _rand((Cout, Cin, KH, KH), torch.float32, 91, 0.1)
    y = F.conv2d(x, w.to(dtype).double(), stride=s, padding=p)
    dy = _rand(y.shape, dtype, 92).double()
    (ref,) = torch.autograd.grad(y, x, dy)
    dys = dy.permute(0, 2, 3, 1).contiguous().to(dtype).to(DEV)
    wt = K.weight_prep(w.to(DEV), Cin, dtype, transposed=True)
    dx = K.conv_dgrad(dys, wt, N, H, W, Cin, Cout, KH, KH, s, p)
    _close(dx.permute(0, 3, 1, 2), ref, dtype, "conv dgrad (>= 64 Ki rows)")


# the 256 x 256-tile engine (igemm256.hip) against the 128 x 128 engine: (kind, shape). Dense GEMMs (M, N, K) with
# ragged M / N, 3x3 im2col convs and TSM 1x1 convs (N frames, H, W, C, Cout), each large enough for >= 128 tiles
G256_CASES = [("dense", (8192 + 77, 2048 + 8, 320)), ("dense", (8192, 3072, 768)),
              ("conv3x3", (64, 28, 28, 128, 512)), ("conv3x3", (1024, 7, 7, 512, 512)),
              ("conv1x1_tsm", (64, 14, 14, 1024, 1024))]


@pytest.mark.parametrize("case", G256_CASES)
def test_gemm256_vs_128(K, case, monkeypatch):
    """VCG_G256=1 / 2 (four / two MFMA phases per k-step) against VCG_G256=0 (the 128 x 128 engine): outputs bit for
    bit (same products, same k order, fp32 accumulation, one rounding); for the convs also the BN statistics
    through bn_finalize (different row partials: to float rounding). The unset default routes the layer-4 3x3
    forward with statistics (the 1024-frame case) to the 256 engine."""
    kind, shp = case
    dt = torch.bfloat16
    outs = {}
    for mode in ("0", "1", "2"):
        monkeypatch.setenv("VCG_G256", mode)
        if kind == "dense":
            M, N, Kd = shp
            A = _rand((M, Kd), dt, 81).to(DEV)
            B = _rand((N, Kd), dt, 82, 0.05).to(DEV)
            outs[mode] = (K.gemm(A, B, M, N, Kd, Kd, Kd), None)
        else:
            Nf, H, W, C, Co = shp
            k, pad = (3, 1) if kind == "conv3x3" else (1, 0)
            T, fold = (16, C // 8) if kind == "conv1x1_tsm" else (0, 0)
            x = _rand((Nf, H, W, C), dt, 83).to(DEV)
            w = K.weight_prep(_rand((Co, C, k, k), torch.float32, 84, 0.05).to(DEV), C, dt)
            M = Nf * H * W
            st = K.stats_buffer(Co, M, DEV)
            y = K.conv_fwd(x, w, Nf, H, W, C, Co, k, k, 1, pad, T, fold, stats=st)
            fin = [torch.empty(Co, device=DEV) for _ in range(4)]
            K.bn_finalize(st, st.shape[1], M, Co, None, None, *fin, None, None, 0.1, 1e-5)
            outs[mode] = (y, (fin[0].double(), fin[1].double()))
        torch.cuda.synchronize()
    ref, rst = outs["0"]
    for mode in ("1", "2"):
        y, st = outs[mode]
        assert torch.equal(y.view(torch.int16), ref.view(torch.int16)), \
            f"VCG_G256={mode}: max {(y.float() - ref.float()).abs().max().item():.3e}"
        if st is not None:
            assert ((st[0] - rst[0]).abs() * rst[1]).max().item() < 1e-5
            assert ((st[1] - rst[1]).abs() / rst[1]).max().item() < 1e-5


# conv1 input gradients whose epilogue also forms the previous block's P = g^T a2 (mask bits, no y):
# (N, H, W, C, Cout, T, res_stride, a2 columns)
P_CASES = [(16, 56, 56, 256, 64, 8, 1, 64), (16, 56, 56, 256, 128, 8, 2, 64), (5, 56, 56, 256, 64, 5, 1, 64),
           (3, 28, 28, 256, 128, 3, 2, 64)]


@pytest.mark.parametrize("case", P_CASES)
def test_conv_dgrad_bwd_p_product(K, case):
    """vcg_conv_dgrad_bwd with a2: g and sum g exactly those of the call without it, and pg = g^T a2 against float64
    as close as the weight-gradient GEMM it replaces (trunk.py: bn3's sum_gx of a layer-1 block whose y3 is not
    stored); a2 of 128 columns is refused (VCG_ERR_UNSUPPORTED -> done False, g still computed)."""
    N, H, W, C, Cout, T, rs, PJ = case
    dt = torch.bfloat16
    dy = _rand((N, H, W, Cout), dt, 91).to(DEV)
    wt = K.weight_prep(_rand((Cout, C, 1, 1), torch.float32, 92, 0.1).to(DEV), C, dt, transposed=True)
    res = _rand((N, (H + 1) // 2, (W + 1) // 2, C) if rs == 2 else (N, H, W, C), dt, 93).to(DEV)
    _, bits = K.bn_apply(_rand((N, H, W, C), dt, 94).to(DEV), torch.ones(C, device=DEV), torch.zeros(C, device=DEV),
                         C, relu=True, bits=True)
    a2 = torch.relu(_rand((N, H, W, PJ), torch.float32, 95)).to(dt).to(DEV)
    mean, inv = torch.zeros(C, device=DEV), torch.ones(C, device=DEV)
    kw = dict(tsm_T=T, tsm_fold=C // 8, res=res, res_stride=rs, bits=bits, mean=mean, invstd=inv)
    s0 = torch.zeros((2, C), device=DEV)
    g0 = K.conv_dgrad_bwd(dy, wt, N, H, W, C, Cout, 1, 1, 1, 0, sums=s0, **kw)
    s1 = torch.zeros((2, C), device=DEV)
    pg = torch.empty((C, PJ), device=DEV)
    g1, done = K.conv_dgrad_bwd(dy, wt, N, H, W, C, Cout, 1, 1, 1, 0, sums=s1, a2=a2, pg=pg, **kw)
    assert done, "the streaming kernel must take the P product at this shape"
    M = N * H * W
    ref_gemm = torch.empty((C, PJ, 1, 1), device=DEV)
    K.conv_wgrad(a2, g1, ref_gemm, N, H, W, PJ, PJ, C, 1, 1, 1, 0, accumulate=False)
    torch.cuda.synchronize()
    assert torch.equal(g0, g1)
    assert (s0[0].double() - s1[0].double()).abs().max().item() <= 1e-4 * (s0[0].abs().max().item() + 1.0)
    ref = g1.view(M, C).double().t() @ a2.view(M, PJ).double()
    sc = ref.abs().max().item() + 1e-6
    e_p = (pg.double() - ref).abs().max().item() / sc
    e_g = (ref_gemm.view(C, PJ).double() - ref).abs().max().item() / sc
    assert e_p <= max(2.0 * e_g, 1e-5), (e_p, e_g)
    a2w = torch.relu(_rand((N, H, W, 128), torch.float32, 96)).to(dt).to(DEV)
    g2, done2 = K.conv_dgrad_bwd(dy, wt, N, H, W, C, Cout, 1, 1, 1, 0, sums=torch.zeros((2, C), device=DEV), a2=a2w,
                                 pg=torch.empty((C, 128), device=DEV), **kw)
    assert not done2 and torch.equal(g2, g0)
