"""The LDS-patch 3x3 convolution (igemm_fast.hip conv3x3_patch_kernel: 3x3 / stride 1 / pad 1 over C = 64, the
layer-1 conv2 of the trunk) against float64 torch and against the im2col engine it replaces.

Both engines accumulate the same bf16 products tap by tap with the same MFMA instruction and operand layout,
so their outputs must be bit-identical; VCG_NO_PATCH=1 (read per call) routes a call to the im2col engine.
"""
import os

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

DEV = "cuda"
BF = torch.bfloat16

# N, H, W, Cout: R rows per tile = 2 (56x56, the trunk's shape), 4 (28x28), 7 (14x14), 9 (9x13, TM = 117),
# 1 (5x72: one row per tile), 7 (7x5), and 128 output channels (two N-tiles)
CASES = [(4, 56, 56, 64), (3, 28, 28, 64), (5, 14, 14, 64), (2, 9, 13, 64), (2, 5, 72, 64), (3, 7, 5, 64),
         (2, 28, 28, 128)]


@pytest.fixture(scope="module")
def K():
    from vcg_hip import _lib, ops
    _lib.call("vcg_init", 0)
    return ops


def _rand(shape, seed, scale=1.0, off=0.0):
    g = torch.Generator().manual_seed(seed)
    return (torch.randn(shape, generator=g) * scale + off).to(BF)


def _both(fn):
    """fn() on the patch engine and on the im2col engine (VCG_NO_PATCH=1)."""
    a = fn()
    os.environ["VCG_NO_PATCH"] = "1"
    try:
        b = fn()
    finally:
        del os.environ["VCG_NO_PATCH"]
    torch.cuda.synchronize()
    return a, b


def _close(out, ref, what):
    out, ref = out.double().cpu(), ref.double().cpu()
    scale = ref.abs().max().item() + 1e-6
    err = (out - ref).abs().max().item()
    assert err <= 2e-2 * scale, f"{what}: max err {err:.3e} vs scale {scale:.3e}"


@pytest.mark.parametrize("case", CASES)
def test_patch_fwd_stats(K, case):
    N, H, W, Cout = case
    C = 64
    x = _rand((N, H, W, C), 1, off=0.5)
    w = _rand((Cout, C, 3, 3), 2, 0.05)
    xs = x.to(DEV)
    wd = K.weight_prep(w.float().to(DEV), C, BF)
    M = N * H * W

    def run():
        st = K.stats_buffer(Cout, M, DEV)
        y = K.conv_fwd(xs, wd, N, H, W, C, Cout, 3, 3, 1, 1, stats=st)
        mean, invstd, scale, shift = (torch.empty(Cout, device=DEV) for _ in range(4))
        K.bn_finalize(st, K.stats_tiles(M), M, Cout, None, None, mean, invstd, scale, shift, None, None, 0.1, 1e-5)
        return y, st, mean, invstd

    (y, st, mean, inv), (y0, _, mean0, inv0) = _both(run)
    assert torch.equal(y, y0), "patch conv != im2col conv"
    ref = F.conv2d(x.double().permute(0, 3, 1, 2), w.double(), padding=1).permute(0, 2, 3, 1)
    _close(y, ref, "patch conv fwd")
    assert float(st[Cout, :, 0].sum()) == M  # slot row counts cover every row once
    yd = y.double().cpu().reshape(M, Cout)
    mu, var = yd.mean(0), yd.var(0, unbiased=False)
    assert torch.allclose(mean.double().cpu(), mu, rtol=1e-5, atol=1e-5)
    assert torch.allclose(inv.double().cpu(), 1 / torch.sqrt(var + 1e-5), rtol=2e-4)
    assert torch.allclose(mean, mean0, rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("case", CASES)
def test_patch_dgrad(K, case):
    N, H, W, C = case  # dx channels C; the gathered dy has Cout = 64
    Cout = 64
    dy = _rand((N, H, W, Cout), 3)
    w = _rand((Cout, C, 3, 3), 4, 0.05)
    wt = K.weight_prep(w.float().to(DEV), C, BF, transposed=True)
    dys = dy.to(DEV)
    dx, dx0 = _both(lambda: K.conv_dgrad(dys, wt, N, H, W, C, Cout, 3, 3, 1, 1))
    assert torch.equal(dx, dx0), "patch dgrad != im2col dgrad"
    xr = torch.zeros((N, C, H, W), dtype=torch.float64, requires_grad=True)
    yr = F.conv2d(xr, w.double(), padding=1)
    (ref,) = torch.autograd.grad(yr, xr, dy.double().permute(0, 3, 1, 2))
    _close(dx, ref.permute(0, 2, 3, 1), "patch dgrad")


@pytest.mark.parametrize("case", [(4, 56, 56, 64), (2, 9, 13, 64), (2, 28, 28, 128)])
def test_patch_dgrad_bwd_affine(K, case):
    """The trunk's fused conv2 input gradient (EPI_BWD_AFF: BN1 ReLU mask from y, BN1 backward sums) on the
    patch engine == the im2col engine, bit for bit (g and the reductions)."""
    N, H, W, C = case
    Cout = 64
    dy = _rand((N, H, W, Cout), 5).to(DEV)
    w = _rand((Cout, C, 3, 3), 6, 0.05).float().to(DEV)
    wt = K.weight_prep(w, C, BF, transposed=True)
    y = _rand((N, H, W, C), 7).to(DEV)
    g0 = torch.Generator().manual_seed(8)
    mean = (torch.randn(C, generator=g0) * 0.1).to(DEV)
    inv = (torch.rand(C, generator=g0) + 0.5).to(DEV)
    msc = (torch.rand(C, generator=g0) + 0.5).to(DEV)
    msh = (torch.randn(C, generator=g0) * 0.2).to(DEV)

    def run():
        sums = torch.zeros((2, C), device=DEV)
        dg, db = torch.zeros(C, device=DEV), torch.zeros(C, device=DEV)
        g = K.conv_dgrad_bwd(dy, wt, N, H, W, C, Cout, 3, 3, 1, 1, y=y, mean=mean, invstd=inv, mscale=msc,
                             mshift=msh, sums=sums, dgamma=dg, dbeta=db)
        return g, sums, dg, db

    (g, sums, dg, db), (g0_, sums0, dg0, db0) = _both(run)
    assert g is not None and torch.equal(g, g0_), "patch fused dgrad != im2col fused dgrad"
    gd = g.double().reshape(-1, C)
    sg = gd.sum(0)
    sx = (gd * (y.double().reshape(-1, C) - mean.double()) * inv.double()).sum(0)
    tol = lambda r: 1e-4 * (r.abs().max().item() + 1.0)  # noqa: E731
    assert (sums[0].double() - sg).abs().max().item() <= tol(sg)
    assert (sums[1].double() - sx).abs().max().item() <= tol(sx)
    assert (db.double() - sg).abs().max().item() <= tol(sg)
    assert (dg.double() - sx).abs().max().item() <= tol(sx)
    # same partial sums, different slot partition: equal to f32 rounding
    assert torch.allclose(sums, sums0, rtol=1e-5, atol=1e-4)


@pytest.mark.parametrize("shape", [(2, 16, 16), (3, 17, 22), (4, 64, 64), (2, 224, 224), (3, 30, 46)])
def test_stem_patch(K, shape):
    """The pair-packed 7x7 / 2 stem on the LDS-patch kernel (stem_patch_kernel) == the im2col engine bit for bit
    (values), BN statistics to f32 rounding, and == float64 torch within bf16 tolerance."""
    N, H, W = shape
    Cin, Cout, k, s, p = 3, 64, 7, 2, 3
    x = _rand((N, Cin, H, W), 21).double()
    w = _rand((Cout, Cin, k, k), 22, 0.1)
    xs = torch.zeros((N, H, W, 4), dtype=BF)
    xs[..., :Cin] = x.permute(0, 2, 3, 1).to(BF)
    xs = xs.to(DEV)
    wd = K.weight_prep(w.float().to(DEV), 4, BF, pair_pad=p)
    OH, OW = K.conv_out_hw(H, W, k, k, s, p)
    M = N * OH * OW

    def run():
        st = K.stats_buffer(Cout, M, DEV)
        y = K.conv_fwd(xs, wd, N, H, W, 4, Cout, k, k, s, p, 0, 0, stats=st)
        mean, invstd, scale, shift = (torch.empty(Cout, device=DEV) for _ in range(4))
        K.bn_finalize(st, K.stats_tiles(M), M, Cout, None, None, mean, invstd, scale, shift, None, None, 0.1, 1e-5)
        return y, st, mean, invstd

    (y, st, mean, inv), (y0, _, mean0, inv0) = _both(run)
    assert torch.equal(y, y0), "stem patch != stem im2col"
    assert float(st[Cout, :, 0].sum()) == M
    assert torch.allclose(mean, mean0, rtol=1e-5, atol=1e-6) and torch.allclose(inv, inv0, rtol=1e-4)
    ref = F.conv2d(x, w.to(BF).double(), stride=s, padding=p).permute(0, 2, 3, 1)
    _close(y, ref, "stem patch fwd")
