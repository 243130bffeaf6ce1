"""The batch-statistics BN backward folded into the consuming 1x1 conv's gradients (vcg_bn_bwd_fold_weights,
vcg_conv_dgrad_bwd_bnfold, vcg_conv_wgrad_bnfold) against the unfused path (vcg_bn_bwd_apply -> the conv's dgrad /
wgrad) and a float64 reference of the same math (torch BatchNorm2d autograd, the bn3 -> conv3 step of the trunk
backward). The fold rounds the scaled weights A w / B w to bf16 where the unfused path rounds dy: the two differ by
rounding only, so the test bounds the fold's error against float64 by a small multiple of the unfused path's."""
import pytest
import torch

from vcg_hip import _lib, ops

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _init():
    _lib.call("vcg_init", 0)


def _bf(t):
    return t.to(torch.bfloat16).to(DEV)


def _case(N, H, W, C, Cout, seed, ymean=0.7):
    """g, y (bf16 [M, Cout]), BN params / sums of y, conv weight w [Cout, C] (fp32), wt [C, Cout] bf16, and the
    epilogue's bn2 (y2 [M, C], mean2, invstd2, scale / shift of its ReLU decision)."""
    gen = torch.Generator().manual_seed(seed)
    M = N * H * W
    g = torch.randn(M, Cout, generator=gen) * 0.02
    g = torch.where(torch.rand(M, Cout, generator=gen) < 0.5, g, torch.zeros_like(g))  # a ReLU-masked gradient
    y = torch.randn(M, Cout, generator=gen) * (0.5 + torch.rand(Cout, generator=gen)) + ymean * torch.randn(Cout, generator=gen)
    gb, yb = _bf(g), _bf(y)
    yd = yb.double()
    mean = yd.mean(0)
    var = yd.var(0, unbiased=False)
    invstd = (var + 1e-5).rsqrt()
    gamma = 0.5 + torch.rand(Cout, generator=gen).double()
    sum_g = gb.double().sum(0)
    sum_gx = (gb.double() * (yd - mean) * invstd).sum(0)
    w = torch.randn(Cout, C, generator=gen) * (1.0 / Cout ** 0.5)
    wt = _bf(w.t().contiguous())
    y2c = (torch.randn(M, C, generator=gen) + 0.3).to(torch.bfloat16)
    m2 = y2c.double().mean(0)
    is2 = (y2c.double().var(0, unbiased=False) + 1e-5).rsqrt()
    y2 = y2c.to(DEV)
    gam2 = 0.5 + torch.rand(C, generator=gen).double()
    bet2 = torch.randn(C, generator=gen).double() * 0.1
    sc2 = (gam2 * is2)
    sh2 = bet2 - m2 * sc2
    f = lambda t: t.float().to(DEV)
    return dict(M=M, g=gb, y=yb, mean=f(mean), invstd=f(invstd), gamma=f(gamma), sum_g=f(sum_g), sum_gx=f(sum_gx),
                wt=wt, y2=y2, mean2=f(m2), invstd2=f(is2), sc2=f(sc2), sh2=f(sh2))


def _dy_ref(c):
    """float64 dy = A g + B y + Cc (the batch-stat BN backward of the masked gradient g)."""
    g, y = c["g"].double(), c["y"].double()
    A = c["gamma"].double() * c["invstd"].double()
    B = -A * c["invstd"].double() * c["sum_gx"].double() / c["M"]
    Cc = -A * c["sum_g"].double() / c["M"] - B * c["mean"].double()
    return A * g + B * y + Cc


SHAPES = [(4, 28, 28, 64, 256), (8, 14, 14, 256, 1024), (3, 7, 9, 128, 512), (2, 7, 7, 512, 2048)]


@pytest.mark.parametrize("shape", SHAPES)
def test_bnfold_dgrad(shape):
    N, H, W, C, Cout = shape
    c = _case(N, H, W, C, Cout, 1)
    M = c["M"]
    wfold, bias = ops.bn_bwd_fold_weights(c["wt"], C, Cout, c["mean"], c["invstd"], c["gamma"], c["sum_g"],
                                          c["sum_gx"], M)
    kw = dict(y=c["y2"], mean=c["mean2"], invstd=c["invstd2"], mscale=c["sc2"], mshift=c["sh2"])
    s_f = torch.zeros(2, C, device=DEV)
    gf = ops.conv_dgrad_bwd_bnfold(c["g"], c["y"], wfold, bias, N, H, W, C, Cout, sums=s_f, **kw)
    assert gf is not None
    # unfused: bn_bwd_apply (dy rounded to bf16) -> fused dgrad with the same epilogue
    dy = ops.bn_bwd_apply(c["g"], None, c["y"], c["mean"], c["invstd"], c["gamma"], c["sum_g"], c["sum_gx"], Cout,
                          train_stats=True)
    s_u = torch.zeros(2, C, device=DEV)
    gu = ops.conv_dgrad_bwd(dy, c["wt"], N, H, W, C, Cout, 1, 1, 1, 0, sums=s_u, **kw)
    torch.cuda.synchronize()
    gf, gu = gf.view(M, C), gu.view(M, C)
    ref = _dy_ref(c) @ c["wt"].double().t()
    keep = (c["y2"].double() * c["sc2"].double() + c["sh2"].double()) > 0
    ref = torch.where(keep, ref, torch.zeros_like(ref))
    scale = ref.abs().max().item()
    ef = (gf.double() - ref).abs().max().item() / scale
    eu = (gu.double() - ref).abs().max().item() / scale
    assert ef < max(2.0 * eu, 8e-3), (ef, eu)
    assert ((gf.double() - ref).abs().mean() / ref.abs().mean()).item() < 8e-3
    assert (gf[~keep] == 0).all()
    # the sums against y2 of the stored gradient (what bn2's backward consumes)
    sref = torch.stack([gf.double().sum(0), (gf.double() * (c["y2"].double() - c["mean2"].double())
                                              * c["invstd2"].double()).sum(0)])
    assert (s_f.double() - sref).abs().max().item() < 1e-3 * (sref.abs().max().item() + 1)


@pytest.mark.parametrize("shape", SHAPES)
def test_bnfold_wgrad(shape):
    N, H, W, C, Cout = shape
    c = _case(N, H, W, C, Cout, 2)
    M = c["M"]
    x = torch.relu(c["y2"])  # a post-ReLU activation (the conv's input)
    cs = torch.zeros(C, device=DEV)
    ops.colsum(x, C, M, C, cs, accumulate=False)
    dw_f = torch.full((Cout, C), 0.25, device=DEV)  # accumulate onto an existing gradient
    ok = ops.conv_wgrad_bnfold(x, c["g"], c["y"], c["mean"], c["invstd"], c["gamma"], c["sum_g"], c["sum_gx"], M, cs,
                               dw_f, N, H, W, C, Cout)
    assert ok
    dy = ops.bn_bwd_apply(c["g"], None, c["y"], c["mean"], c["invstd"], c["gamma"], c["sum_g"], c["sum_gx"], Cout,
                          train_stats=True)
    dw_u = torch.full((Cout, C, 1, 1), 0.25, device=DEV)
    ops.conv_wgrad(x, dy, dw_u, N, H, W, C, C, Cout, 1, 1, 1, 0)
    torch.cuda.synchronize()
    ref = _dy_ref(c).t() @ x.double() + 0.25
    d = ref - 0.25
    scale = d.abs().max().item()
    ef = (dw_f.double() - ref).abs().max().item() / scale
    eu = (dw_u.view(Cout, C).double() - ref).abs().max().item() / scale
    assert ef < max(2.0 * eu, 2e-3), (ef, eu)


def test_bnfold_deterministic():
    N, H, W, C, Cout = 8, 14, 14, 256, 1024
    c = _case(N, H, W, C, Cout, 3)
    M = c["M"]
    outs = []
    for _ in range(2):
        wfold, bias = ops.bn_bwd_fold_weights(c["wt"], C, Cout, c["mean"], c["invstd"], c["gamma"], c["sum_g"],
                                              c["sum_gx"], M)
        s = torch.zeros(2, C, device=DEV)
        gf = ops.conv_dgrad_bwd_bnfold(c["g"], c["y"], wfold, bias, N, H, W, C, Cout, y=c["y2"], mean=c["mean2"],
                                       invstd=c["invstd2"], mscale=c["sc2"], mshift=c["sh2"], sums=s)
        x = torch.relu(c["y2"])
        cs = torch.zeros(C, device=DEV)
        ops.colsum(x, C, M, C, cs, accumulate=False)
        dw = torch.zeros(Cout, C, device=DEV)
        ops.conv_wgrad_bnfold(x, c["g"], c["y"], c["mean"], c["invstd"], c["gamma"], c["sum_g"], c["sum_gx"], M, cs,
                              dw, N, H, W, C, Cout)
        outs.append((gf, s, dw, bias))
    torch.cuda.synchronize()
    for a, b in zip(*outs):
        assert torch.equal(a, b)


@pytest.mark.parametrize("rows,N", [(3211264 // 8, 64), (200704, 256), (50176 + 37, 512), (802816, 128)])
def test_colsum_tall(rows, N):
    """vcg_colsum on the trunk's tall conv inputs (the fold's colsum(x)): fixed-order partials, vs float64."""
    gen = torch.Generator().manual_seed(rows + N)
    x = (torch.randn(rows, N, generator=gen) + 0.5).to(torch.bfloat16).to(DEV)
    out = torch.full((N,), 2.0, device=DEV)
    ops.colsum(x, N, rows, N, out, accumulate=True)
    torch.cuda.synchronize()
    ref = x.double().sum(0) + 2.0
    assert ((out.double() - ref).abs() / ref.abs().clamp_min(1.0)).max().item() < 1e-5
    out2 = torch.zeros(N, device=DEV)
    ops.colsum(x, N, rows, N, out2, accumulate=False)
    out3 = torch.zeros(N, device=DEV)
    ops.colsum(x, N, rows, N, out3, accumulate=False)
    torch.cuda.synchronize()
    assert torch.equal(out2, out3)


@pytest.mark.parametrize("shape", [(4, 28, 28, 64, 256), (3, 7, 9, 128, 512), (8, 14, 14, 256, 1024)])
def test_conv1x1_bn_res_relu(shape):
    """bn3 + identity + ReLU as a second conv3 GEMM pass (vcg_conv1x1_bn_res_relu) against conv -> bn_apply (the stored
    bf16 y3 read back): one bf16 rounding apart (the GEMM rounds x W' + b instead of y3), mask bits = out > 0."""
    N, H, W, C, Cout = shape
    M = N * H * W
    gen = torch.Generator().manual_seed(7)
    x = _bf(torch.relu(torch.randn(M, C, generator=gen)))
    w = (torch.randn(Cout, C, generator=gen) / C ** 0.5).to(DEV)
    res = _bf(torch.relu(torch.randn(M, Cout, generator=gen)))
    y = x.double() @ w.double().t()
    sc = (0.5 + torch.rand(Cout, generator=gen)).to(DEV) / y.std(0).float()
    sh = (torch.randn(Cout, generator=gen) * 0.3).to(DEV) - y.mean(0).float() * sc
    wf = ops.weight_fold(w, sc, torch.bfloat16)
    r = ops.conv1x1_bn_res_relu(x, wf, sh, res, M, Cout, C)
    assert r is not None
    out, bits = r
    y3 = ops.gemm(x, ops.weight_fold(w, torch.ones(Cout, device=DEV), torch.bfloat16), M, Cout, C, C, C)
    ref, rbits = ops.bn_apply(y3, sc, sh, Cout, relu=True, res=res, bits=True)
    torch.cuda.synchronize()
    exact = torch.relu(y * sc.double() + sh.double() + res.double())
    e_new = (out.double() - exact).abs().max().item()
    e_old = (ref.double() - exact).abs().max().item()
    assert e_new <= max(1.5 * e_old, 3e-2 * exact.abs().max().item()), (e_new, e_old)
    # bits: byte (m Cout + n) / 8, bit n % 8 = out > 0 of this pass
    pos = (out.view(-1, 8) > 0).to(torch.uint8)
    expect = (pos * (2 ** torch.arange(8, device=DEV, dtype=torch.uint8))).sum(1).to(torch.uint8)
    assert torch.equal(bits, expect)
    assert (bits != rbits).float().mean().item() < 0.02


def _case_a2(N, H, W, C, Cout, seed):
    """conv3 input a2 [M, C], master weight w3 [Cout, C] f32, its bf16 dgrad operand wt [C, Cout], the stored conv
    output y3 = bf16(a2 bf16(w3)^T) with its batch statistics, a masked upstream gradient g and its BN sums."""
    gen = torch.Generator().manual_seed(seed)
    M = N * H * W
    a2 = _bf(torch.relu(torch.randn(M, C, generator=gen) + 0.2))
    w3 = (torch.randn(Cout, C, generator=gen) / C ** 0.5).to(DEV)
    wt = w3.t().contiguous().to(torch.bfloat16)
    y3 = (a2.double() @ wt.double()).to(torch.bfloat16)
    yd = y3.double()
    mean, invstd = yd.mean(0), (yd.var(0, unbiased=False) + 1e-5).rsqrt()
    g = torch.randn(M, Cout, generator=gen) * 0.02
    g = _bf(torch.where(torch.rand(M, Cout, generator=gen) < 0.5, g, torch.zeros_like(g)))
    gamma = (0.5 + torch.rand(Cout, generator=gen)).to(DEV)
    sum_g = g.double().sum(0)
    sum_gx = (g.double() * (yd - mean) * invstd).sum(0)
    f = lambda t: t.float().to(DEV)
    return dict(M=M, a2=a2, w3=w3, wt=wt, y=y3, g=g, mean=f(mean), invstd=f(invstd), gamma=gamma, sum_g=f(sum_g),
                sum_gx=f(sum_gx))


@pytest.mark.parametrize("shape", [(4, 28, 28, 64, 256), (3, 7, 9, 128, 512), (8, 14, 14, 256, 1024)])
def test_bnfold_a2_dgrad_wgrad(shape):
    """The a2 form of the fold (y3 = a2 w3^T never read): input gradient over [g | a2] and weight gradient from
    g^T a2 and a2^T a2, against float64 of the stored-y3 math and the unfused bn_bwd_apply path."""
    N, H, W, C, Cout = shape
    c = _case_a2(N, H, W, C, Cout, 5)
    M = c["M"]
    cs = torch.zeros(C, device=DEV)
    ops.colsum(c["a2"], C, M, C, cs, accumulate=False)
    wfold, bias = ops.bn_bwd_fold_weights_a2(c["wt"], C, Cout, c["invstd"], c["gamma"], c["sum_g"], c["sum_gx"], M, cs)
    gf = ops.conv_dgrad_bwd_bnfold(c["g"], c["a2"], wfold, bias, N, H, W, C, Cout, Ky=C)
    dy = ops.bn_bwd_apply(c["g"], None, c["y"], c["mean"], c["invstd"], c["gamma"], c["sum_g"], c["sum_gx"], Cout,
                          train_stats=True)
    gu = ops.conv_dgrad(dy, c["wt"], N, H, W, C, Cout, 1, 1, 1, 0)
    Pg = torch.empty(Cout, C, 1, 1, device=DEV)
    G = torch.empty(C, C, 1, 1, device=DEV)
    ops.conv_wgrad(c["a2"], c["g"], Pg, N, H, W, C, C, Cout, 1, 1, 1, 0, accumulate=False)
    ops.conv_wgrad(c["a2"], c["a2"], G, N, H, W, C, C, C, 1, 1, 1, 0, accumulate=False)
    dw_f = torch.full((Cout, C), 0.5, device=DEV)
    ops.bn_bwd_fold_wgrad_a2(Pg.view(Cout, C), G.view(C, C), c["w3"], Cout, C, c["mean"], c["invstd"], c["gamma"],
                             c["sum_g"], c["sum_gx"], M, cs, dw_f)
    dw_u = torch.full((Cout, C, 1, 1), 0.5, device=DEV)
    ops.conv_wgrad(c["a2"], dy, dw_u, N, H, W, C, C, Cout, 1, 1, 1, 0)
    torch.cuda.synchronize()
    A = c["gamma"].double() * c["invstd"].double()
    B = -A * c["invstd"].double() * c["sum_gx"].double() / M
    Cc = -A * c["sum_g"].double() / M - B * c["mean"].double()
    dy_ref = A * c["g"].double() + B * c["y"].double() + Cc
    ref = dy_ref @ c["wt"].double().t()
    sc = ref.abs().max().item()
    ef = (gf.view(M, C).double() - ref).abs().max().item() / sc
    eu = (gu.view(M, C).double() - ref).abs().max().item() / sc
    assert ef < max(2.0 * eu, 8e-3), (ef, eu)
    wref = dy_ref.t() @ c["a2"].double()
    wsc = wref.abs().max().item()
    ewf = (dw_f.double() - 0.5 - wref).abs().max().item() / wsc
    ewu = (dw_u.view(Cout, C).double() - 0.5 - wref).abs().max().item() / wsc
    assert ewf < max(2.0 * ewu, 5e-3), (ewf, ewu)


def test_conv1x1_stats_matches_stored():
    """Statistics-only conv3 GEMM (y3 never stored) == the storing conv's statistics, bit for bit."""
    N, H, W, C, Cout = 4, 28, 28, 64, 256
    M = N * H * W
    gen = torch.Generator().manual_seed(9)
    x = _bf(torch.relu(torch.randn(M, C, generator=gen)))
    w = _bf(torch.randn(Cout, C, generator=gen) / C ** 0.5)
    s1, s2 = ops.stats_buffer(Cout, M, DEV), ops.stats_buffer(Cout, M, DEV)
    ops.conv_fwd(x.view(N, H, W, C), w, N, H, W, C, Cout, 1, 1, 1, 0, stats=s1)
    assert ops.conv1x1_stats(x, w, s2, M, Cout, C)
    outs = []
    for st in (s1, s2):
        mean, inv, sc, sh = (torch.empty(Cout, device=DEV) for _ in range(4))
        ops.bn_finalize(st, ops.stats_tiles(M), M, Cout, torch.ones(Cout, device=DEV), torch.zeros(Cout, device=DEV),
                        mean, inv, sc, sh)
        outs.append((mean, inv))
    torch.cuda.synchronize()
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])


@pytest.mark.parametrize("shape", [(4, 28, 28, 256, 64, 4), (4, 14, 14, 512, 128, 4), (8, 14, 14, 1024, 256, 4)])
def test_dgrad_bits_only_sums_and_sumgx(shape):
    """The conv1 dgrad epilogue with the mask bits and no y (the previous block's y3 not stored): the same g as with
    y, sum g to float rounding (at K = 256 the bits-only epilogue streams in 64 x 128 tiles while the y form stays on
    the persistent engine: other partial sums), sum_gx written 0; sum_gx from g^T a2 (bn_bwd_sumgx_from_wgrad)
    matches the y3 reduction."""
    N, H, W, C, Co, T = shape
    M = N * H * W
    gen = torch.Generator().manual_seed(11)
    dy = _bf(torch.randn(M, Co, generator=gen) * 0.1)
    wt = _bf(torch.randn(C, Co, generator=gen) / Co ** 0.5)
    res = _bf(torch.randn(M, C, generator=gen) * 0.1)
    planes = C // 4
    a2 = _bf(torch.relu(torch.randn(M, planes, generator=gen)))
    w3 = _bf(torch.randn(C, planes, generator=gen) / planes ** 0.5)  # the previous block's conv3 (forward layout)
    y3 = (a2.double() @ w3.double().t()).to(torch.bfloat16)
    bits = ((torch.rand(M * C // 8, generator=gen) * 255).to(torch.uint8)).to(DEV)
    mean = y3.double().mean(0).float()
    invstd = (y3.double().var(0, unbiased=False) + 1e-5).rsqrt().float()
    fold = C // 8
    outs = []
    for yy in (y3, None):
        sums = torch.zeros(2, C, device=DEV)
        gg = ops.conv_dgrad_bwd(dy.view(N, H, W, Co), wt, N, H, W, C, Co, 1, 1, 1, 0, tsm_T=T, tsm_fold=fold,
                                res=res.view(N, H, W, C), bits=bits, y=None if yy is None else yy.view(N, H, W, C),
                                mean=mean, invstd=invstd, sums=sums)
        outs.append((gg, sums))
    torch.cuda.synchronize()
    (g1, s1), (g2, s2) = outs
    assert torch.equal(g1, g2)
    assert (s1[0].double() - s2[0].double()).abs().max().item() <= 1e-4 * (s1[0].abs().max().item() + 1.0)
    assert (s2[1] == 0).all()
    Pg = torch.empty(C, planes, 1, 1, device=DEV)
    ops.conv_wgrad(a2.view(N, H, W, planes), g2.view(M, C), Pg, N, H, W, planes, planes, C, 1, 1, 1, 0,
                   accumulate=False)
    sgx = torch.empty(C, device=DEV)
    ops.bn_bwd_sumgx_from_wgrad(Pg.view(C, planes), w3, C, planes, mean, invstd, s2[0], sgx)
    torch.cuda.synchronize()
    ref = (g2.view(M, C).double() * (a2.double() @ w3.double().t() - mean.double()) * invstd.double()).sum(0)
    assert (sgx.double() - ref).abs().max().item() < 2e-3 * (ref.abs().max().item() + 1e-3)
    assert (s1[1].double() - ref).abs().max().item() < 2e-2 * (ref.abs().max().item() + 1e-3)


def test_conv1x1_bn_res_relu_affine_residual():
    """A layer's first block: the residual is the downsample BN's output, fma(yd, rs, rb) in the epilogue, against
    conv -> bn_apply(res=yd, rscale, rshift)."""
    N, H, W, C, Cout = 4, 28, 28, 128, 512
    M = N * H * W
    gen = torch.Generator().manual_seed(13)
    x = _bf(torch.relu(torch.randn(M, C, generator=gen)))
    w = (torch.randn(Cout, C, generator=gen) / C ** 0.5).to(DEV)
    yd = _bf(torch.randn(M, Cout, generator=gen) + 0.3)
    sc = (0.5 + torch.rand(Cout, generator=gen)).to(DEV)
    sh = (torch.randn(Cout, generator=gen) * 0.3).to(DEV)
    rs = (0.5 + torch.rand(Cout, generator=gen)).to(DEV)
    rb = (torch.randn(Cout, generator=gen) * 0.3).to(DEV)
    out, bits = ops.conv1x1_bn_res_relu(x, ops.weight_fold(w, sc, torch.bfloat16), sh, yd, M, Cout, C, res_scale=rs,
                                        res_shift=rb)
    y3 = ops.gemm(x, ops.weight_fold(w, torch.ones(Cout, device=DEV), torch.bfloat16), M, Cout, C, C, C)
    ref, rbits = ops.bn_apply(y3, sc, sh, Cout, relu=True, res=yd, rscale=rs, rshift=rb, bits=True)
    torch.cuda.synchronize()
    exact = torch.relu((x.double() @ w.double().t()) * sc.double() + sh.double() + yd.double() * rs.double()
                       + rb.double())
    e_new = (out.double() - exact).abs().max().item()
    e_old = (ref.double() - exact).abs().max().item()
    assert e_new <= max(1.5 * e_old, 3e-2 * exact.abs().max().item()), (e_new, e_old)
    pos = (out.view(-1, 8) > 0).to(torch.uint8)
    assert torch.equal(bits, (pos * (2 ** torch.arange(8, device=DEV, dtype=torch.uint8))).sum(1).to(torch.uint8))
    assert (bits != rbits).float().mean().item() < 0.02


@pytest.mark.parametrize("rows,C", [(3211264 // 4, 64), (802816 // 2 + 13, 128), (200704, 256), (50176, 512)])
def test_bn_apply_colsum(rows, C):
    """bn_apply + the column sums of its stored output in one pass == bn_apply (bit for bit) and colsum."""
    gen = torch.Generator().manual_seed(rows % 97 + C)
    y = _bf(torch.randn(rows, C, generator=gen))
    sc = (0.5 + torch.rand(C, generator=gen)).to(DEV)
    sh = (torch.randn(C, generator=gen) * 0.2).to(DEV)
    a, cs = ops.bn_apply_colsum(y, sc, sh, C)  # (the trunk's bn2 apply where the Gram pass does not apply)
    ref = ops.bn_apply(y, sc, sh, C, relu=True)
    csr = torch.zeros(C, device=DEV)
    ops.colsum(ref, C, rows, C, csr, accumulate=False)
    torch.cuda.synchronize()
    assert torch.equal(a, ref)
    assert ((cs.double() - csr.double()).abs() / csr.double().abs().clamp_min(1.0)).max().item() < 1e-5


@pytest.mark.parametrize("rows,C", [(3211264 // 4 + 5, 64), (802816 // 2 + 13, 128), (200704, 256), (77, 64)])
def test_bn_apply_gram(rows, C):
    """bn_apply + colsum + the Gram matrix a^T a of the stored output in one pass: a == bn_apply bit for bit, colsum
    and gram against float64 sums of the same bf16 values, deterministic; ragged row counts (tail rows contribute
    nothing). The channels whose BN shift dominates (beta > 6 |gamma|) are accumulated centred (bn_gram.hip): the
    rebuilt uncentred Gram is as exact as the plain one (fp32 MFMA accumulation: ~1e-6 relative)."""
    gen = torch.Generator().manual_seed(rows % 89 + C)
    y = _bf(torch.randn(rows, C, generator=gen) + 0.2)
    sc = (0.5 + torch.rand(C, generator=gen)).to(DEV)
    sh = (torch.randn(C, generator=gen) * 0.2).to(DEV)
    sh[::5] += 12.0  # (every 5th channel centred: beta > 6 |gamma|)
    mean, inv = torch.full((C,), 0.2, device=DEV), torch.ones(C, device=DEV)
    a, cs, G, g64 = ops.bn_apply_gram(y, sc, sh, C, mean, inv)
    ref = ops.bn_apply(y, sc, sh, C, relu=True)
    torch.cuda.synchronize()
    assert torch.equal(a, ref)
    ad = ref.double()
    csr = ad.sum(0)
    Gr = ad.t() @ ad
    assert ((cs.double() - csr).abs() / csr.abs().clamp_min(1.0)).max().item() < 1e-5
    eg = ((G.double() - Gr).abs().max() / Gr.abs().max()).item()
    print(f"gram max err {eg:.2e} of max |G|")
    assert eg < 1e-5
    assert torch.equal(G, G.t())
    c = g64[C * C + C:]
    assert (c[::5] > 0).all() and c.count_nonzero().item() <= (C + 4) // 5 + C // 4
    d = g64[C * C:C * C + C]
    Gc = g64[:C * C].view(C, C)
    Gu = Gc + d[:, None] * c[None, :] + c[:, None] * d[None, :] + rows * c[:, None] * c[None, :]
    assert ((Gu - Gr).abs().max() / Gr.abs().max()).item() < 1e-5
    assert ((d + rows * c - csr).abs() / csr.abs().clamp_min(1.0)).max().item() < 1e-5
    a2, cs2, G2, g642 = ops.bn_apply_gram(y, sc, sh, C, mean, inv)
    assert torch.equal(cs, cs2) and torch.equal(G, G2) and torch.equal(g64, g642)


@pytest.mark.parametrize("M,C,N", [(3211264 // 8, 64, 256), (802816 // 4, 128, 512), (50176, 256, 1024)])
def test_bn_stats_from_gram(M, C, N):
    """conv3's batch statistics from its input's Gram matrix and column sums (bn_stats_from_gram -> bn_finalize)
    against float64 statistics of the exact product x w^T (x >= 0 after the ReLU, w the bf16 GEMM weights): mean and
    invstd within 1e-4 relative; also within bf16 rounding of the statistics of the stored bf16 product (the
    conv1x1_stats path it replaces)."""
    gen = torch.Generator().manual_seed(M % 101 + C)
    y = _bf(torch.randn(M, C, generator=gen))
    sc = (0.5 + torch.rand(C, generator=gen)).to(DEV)
    sh = (torch.randn(C, generator=gen) * 0.3 + 0.2).to(DEV)
    a, cs, G, g64 = ops.bn_apply_gram(y, sc, sh, C, torch.zeros(C, device=DEV), torch.ones(C, device=DEV))
    w = _bf(torch.randn(N, C, generator=gen) * (1.0 / C ** 0.5))
    stats = ops.stats_buffer(N, M, DEV)
    ops.bn_stats_from_gram(g64, w, M, N, C, stats)
    out = [torch.empty(N, device=DEV) for _ in range(4)]
    ops.bn_finalize(stats, stats.shape[1], M, N, None, None, *out, None, None, 0.1, 1e-5)
    st2 = ops.stats_buffer(N, M, DEV)
    assert ops.conv1x1_stats(a, w, st2, M, N, C)
    out2 = [torch.empty(N, device=DEV) for _ in range(4)]
    ops.bn_finalize(st2, ops.stats_tiles(M), M, N, None, None, *out2, None, None, 0.1, 1e-5)
    torch.cuda.synchronize()
    yx = a.double() @ w.double().t()
    mean = yx.mean(0)
    inv = (yx.var(0, unbiased=False) + 1e-5).rsqrt()
    e_mean = ((out[0].double() - mean).abs() / yx.std(0)).max().item()
    e_inv = ((out[1].double() - inv).abs() / inv).max().item()
    print(f"gram stats: mean err {e_mean:.2e} (of std), invstd rel err {e_inv:.2e}; GEMM stats of bf16 y: "
          f"{((out2[0].double() - mean).abs() / yx.std(0)).max().item():.2e}, "
          f"{((out2[1].double() - inv).abs() / inv).max().item():.2e}")
    assert e_mean < 1e-4 and e_inv < 1e-4


@pytest.mark.parametrize("M,C,N", [(3211264 // 8 + 7, 64, 256), (802816 // 4 + 3, 128, 512), (50176 + 9, 256, 1024),
                                   (5, 64, 256)])
def test_conv1x1_bn_res_relu_streaming_vs_persistent(monkeypatch, M, C, N):
    """The register-streaming bnres kernel (stream1x1.hip) against the persistent LDS-staged engine (VCG_RS1X1=0):
    bit-identical output and mask bits (same products, order and roundings), ragged row counts included."""
    gen = torch.Generator().manual_seed(M % 113 + C)
    x = _bf(torch.relu(torch.randn(M, C, generator=gen)))
    wf = _bf(torch.randn(N, C, generator=gen) / C ** 0.5)
    bias = (torch.randn(N, generator=gen) * 0.3).to(DEV)
    res = _bf(torch.relu(torch.randn(M, N, generator=gen)) - 0.3)
    out = {}
    for flag in ("0", "1"):
        monkeypatch.setenv("VCG_RS1X1", flag)
        r = ops.conv1x1_bn_res_relu(x, wf, bias, res, M, N, C)
        assert r is not None
        out[flag] = r
    torch.cuda.synchronize()
    assert torch.equal(out["0"][0], out["1"][0])
    assert torch.equal(out["0"][1], out["1"][1])


@pytest.mark.parametrize("M,C,N", [(200704, 64, 256), (50176 + 77, 256, 512)])
def test_bn_stats_from_gram_large_mean(M, C, N):
    """bn3's statistics from the Gram matrix where the a2 channels' |mean| is 30x their std (a2 = relu(0.1 z + 3): the
    BN shift dominates its scale, the ReLU always passes) and y3's 200-450x (all-positive conv3 weights): an uncentred
    fp32 Gram cancels there (E[y^2] - E[y]^2 over channels whose mean^2 is 900x their variance), so such channels are
    accumulated centred at bf16(beta) (bn_gram.hip) and the statistics subtract in double. mean within 1e-4 of std and
    invstd within 1e-4 relative of float64 statistics of the exact product."""
    gen = torch.Generator().manual_seed(M % 97 + C)
    y = _bf(torch.randn(M, C, generator=gen))
    sc = torch.full((C,), 0.1).to(DEV)
    sh = torch.full((C,), 3.0).to(DEV)
    a, cs, G, g64 = ops.bn_apply_gram(y, sc, sh, C, torch.zeros(C, device=DEV), torch.ones(C, device=DEV))
    assert (g64[C * C + C:] == 3.0).all()
    w = _bf(torch.randn(N, C, generator=gen).abs() * (1.0 / C ** 0.5) + 0.05)
    stats = ops.stats_buffer(N, M, DEV)
    ops.bn_stats_from_gram(g64, w, M, N, C, stats)
    out = [torch.empty(N, device=DEV) for _ in range(4)]
    ops.bn_finalize(stats, stats.shape[1], M, N, None, None, *out, None, None, 0.1, 1e-5)
    torch.cuda.synchronize()
    yx = a.double() @ w.double().t()
    mean, std = yx.mean(0), yx.std(0)
    ratio = (mean.abs() / std).min().item()
    inv = (yx.var(0, unbiased=False) + 1e-5).rsqrt()
    e_mean = ((out[0].double() - mean).abs() / std).max().item()
    e_inv = ((out[1].double() - inv).abs() / inv).max().item()
    print(f"large-mean gram stats: |mean| / std >= {ratio:.0f}; mean err {e_mean:.2e} (of std), invstd rel err "
          f"{e_inv:.2e}")
    assert ratio > 30
    assert e_mean < 1e-4 and e_inv < 1e-4


@pytest.mark.parametrize("M,C,N,fold,upd", [(3211264 // 8, 64, 256, True, True), (802816 // 4 + 3, 128, 512, True, False),
                                            (50176, 256, 1024, False, True), (7, 64, 256, True, True),
                                            (100352, 48, 200, True, True)])
def test_bn_finalize_from_gram_vs_three_calls(M, C, N, fold, upd):
    """bn_finalize_from_gram (statistics + finalize + weight fold in one launch) against bn_stats_from_gram ->
    bn_finalize -> weight_fold: bit-identical mean / invstd / scale / shift, running statistics and folded weights
    (the same float roundings of the same double arithmetic); ragged M, N not a multiple of 16 included."""
    gen = torch.Generator().manual_seed(M % 89 + C + N)
    y = _bf(torch.randn(M, C, generator=gen))
    sc = (0.5 + torch.rand(C, generator=gen)).to(DEV)
    sh = (torch.randn(C, generator=gen) * 0.3 + 0.2).to(DEV)
    if C in (64, 128, 256):
        _, _, _, g64 = ops.bn_apply_gram(y, sc, sh, C, torch.zeros(C, device=DEV), torch.ones(C, device=DEV))
    else:  # (C = 48: a synthetic centred Gram record -- the row kernel's C % 16 shapes beyond bn_apply_gram's)
        a = torch.relu(y.float() * sc + sh).double()
        c = torch.zeros(C, dtype=torch.float64, device=DEV)
        g64 = torch.cat([(a.t() @ a).flatten(), a.sum(0), c])
    w32 = (torch.randn(N, C, generator=gen) * (1.0 / C ** 0.5)).to(DEV)
    w = w32.to(torch.bfloat16)
    gamma = (1.0 + 0.2 * torch.randn(N, generator=gen)).to(DEV)
    beta = (0.1 * torch.randn(N, generator=gen)).to(DEV)
    rm0 = torch.randn(N, generator=gen).to(DEV)
    rv0 = (0.5 + torch.rand(N, generator=gen)).to(DEV)
    stats = ops.stats_buffer(N, M, DEV)
    ops.bn_stats_from_gram(g64, w, M, N, C, stats)
    ref = [torch.empty(N, device=DEV) for _ in range(4)]
    rm1, rv1 = rm0.clone(), rv0.clone()
    ops.bn_finalize(stats, stats.shape[1], M, N, gamma, beta, *ref, rm1 if upd else None, rv1 if upd else None,
                    0.1, 1e-5)
    wf_ref = ops.weight_fold(w32, ref[2], torch.bfloat16) if fold else None
    out = [torch.full((N,), float("nan"), device=DEV) for _ in range(4)]
    rm2, rv2 = rm0.clone(), rv0.clone()
    wf = torch.empty((N, C), dtype=torch.bfloat16, device=DEV) if fold else None
    ops.bn_finalize_from_gram(g64, w, M, N, C, gamma, beta, *out, rm2 if upd else None, rv2 if upd else None, 0.1,
                              1e-5, w32 if fold else None, wf)
    torch.cuda.synchronize()
    for r, o in zip(ref, out):
        assert torch.equal(r, o)
    assert torch.equal(rm1, rm2) and torch.equal(rv1, rv2)
    if not upd:
        assert torch.equal(rm2, rm0) and torch.equal(rv2, rv0)
    if fold:
        assert torch.equal(wf_ref, wf)
