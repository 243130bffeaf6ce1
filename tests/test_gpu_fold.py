"""The scoring forward's BN fold (trunk._block_fwd_folded) kernel by kernel, against float64 torch:
vcg_weight_fold, vcg_conv_fwd_bias_act (1x1 + TSM, 3x3 stride 1 and 2, 1x1 stride 2, M not a multiple of 128), and
vcg_gemm with bias + ReLU + residual on the 128- and 64-column tiles with and without VCG_ACT_FLAG_ROUND_PRE; then
folded vs unfolded bf16 bottlenecks on the same input, and the whole trunk (with the fold cache).

Tolerances: bf16 storage, one output rounding (2^-8) plus bf16 operands: 2e-2 of max|ref| per kernel; one folded
bottleneck vs the unfolded one: 2e-2 relative Frobenius error."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _rand(shape, seed, scale=1.0):
    g = torch.Generator().manual_seed(seed)
    return torch.randn(shape, generator=g) * scale


def _close(out, ref, tol, what):
    out, ref = out.detach().double().cpu(), ref.detach().double().cpu()
    err = (out - ref).abs().max().item()
    scale = ref.abs().max().item() + 1e-6
    assert err <= tol * scale, f"{what}: max err {err:.3e} vs scale {scale:.3e}"


@pytest.fixture(scope="module")
def K():
    from vcg_hip import _lib, ops
    _lib.call("vcg_init", 0)
    return ops


def test_weight_fold_bitexact(K):
    w = _rand((96, 64 * 9), 1).to(DEV)
    sc = (torch.rand(96, generator=torch.Generator().manual_seed(2)) + 0.5).to(DEV)
    got = K.weight_fold(w, sc, torch.bfloat16)
    assert torch.equal(got, (w * sc[:, None]).to(torch.bfloat16))
    got32 = K.weight_fold(w, sc, torch.float32)
    assert torch.equal(got32, w * sc[:, None])


def _tsm_ref(x, T, fold):
    nt, c, h, w = x.shape
    x = x.view(nt // T, T, c, h, w)
    out = torch.zeros_like(x)
    out[:, :-1, :fold] = x[:, 1:, :fold]
    out[:, 1:, fold:2 * fold] = x[:, :-1, fold:2 * fold]
    out[:, :, 2 * fold:] = x[:, :, 2 * fold:]
    return out.view(nt, c, h, w)


FOLD_CASES = [
    # N, H, W, Cin, Cout, K, stride, pad, tsm_T, act
    (8, 14, 14, 64, 64, 1, 1, 0, 4, 1),      # conv1 + TSM gather, ReLU
    (4, 56, 56, 64, 64, 3, 1, 1, 0, 1),      # layer-1 conv2 shape (the patch kernel's; bias epilogue -> im2col)
    (4, 15, 13, 128, 128, 3, 2, 1, 0, 1),    # stride-2 conv2, odd sizes
    (4, 14, 14, 256, 512, 1, 2, 0, 0, 0),    # downsample 1x1/2, no activation
    (3, 7, 7, 512, 256, 1, 1, 0, 0, 1),      # M = 147: ragged last tile
    (2, 9, 11, 64, 128, 3, 1, 1, 0, 1),      # 64 <-> 128 columns, M = 198
]


@pytest.mark.parametrize("case", FOLD_CASES)
def test_conv_fwd_bias_act(K, case):
    N, H, W, Cin, Cout, KS, s, p, T, act = case
    x = _rand((N, Cin, H, W), 3).to(torch.bfloat16).double()
    w = _rand((Cout, Cin, KS, KS), 4, 0.05)
    bias = _rand((Cout,), 5)
    fold = Cin // 8 if T else 0
    xin = _tsm_ref(x, T, fold) if T else x
    ref = F.conv2d(xin, w.to(torch.bfloat16).double(), stride=s, padding=p) + bias.double()[None, :, None, None]
    if act:
        ref = ref.clamp_min(0)
    xs = x.permute(0, 2, 3, 1).to(torch.bfloat16).contiguous().to(DEV)
    wd = K.weight_prep(w.to(DEV), Cin, torch.bfloat16)
    y = K.conv_fwd_bias_act(xs, wd, bias.to(DEV), act, N, H, W, Cin, Cout, KS, KS, s, p, T, fold)
    _close(y.permute(0, 3, 1, 2), ref, 2e-2, f"conv_fwd_bias_act {case}")


@pytest.mark.parametrize("N", [128, 64])
@pytest.mark.parametrize("round_pre", [False, True])
@pytest.mark.parametrize("M", [300, 1024])
def test_gemm_bias_relu_residual(K, N, round_pre, M):
    Kd = 256
    A = _rand((M, Kd), 6).to(torch.bfloat16)
    B = _rand((N, Kd), 7, 0.06).to(torch.bfloat16)
    bias = _rand((N,), 8)
    R = _rand((M, N), 9).to(torch.bfloat16)
    pre = A.double() @ B.double().T + bias.double()
    if round_pre:
        pre = pre.to(torch.bfloat16).double()
    ref = (pre + R.double()).clamp_min(0)
    act = K.ACT_RELU | (K.ACT_FLAG_ROUND_PRE if round_pre else 0)
    out = K.gemm(A.to(DEV), B.to(DEV), M, N, Kd, Kd, Kd, bias=bias.to(DEV), act=act, residual=R.to(DEV), ldr=N)
    _close(out, ref, 2e-2, f"gemm bias+relu+res N={N} round={round_pre}")


BLOCKS = [(1, 0, 28, 64), (1, 2, 28, 256), (2, 0, 28, 256), (3, 1, 7, 1024), (4, 0, 7, 1024), (4, 2, 4, 2048)]


@pytest.mark.parametrize("blk_at", BLOCKS)
def test_folded_block_matches_unfolded(blk_at):
    """One bottleneck of the bf16 scoring forward with its BNs folded (conv1 + TSM gather and conv2 with bias + ReLU,
    the downsample conv with bias, conv3 as one GEMM with residual, bias, ReLU and the ROUND_PRE rounding) against the
    unfolded bf16 block (conv, running-stat BN apply passes) on the same input, with non-trivial running statistics
    and affine parameters. Frames N = 12 (3 clips of 4): ragged M in layers 3 / 4. A single block has no depth over
    which BN can amplify rounding (the whole random-init trunk does: see below), so the bar is the bf16 rounding of
    three convs: 2e-2 relative (Frobenius), 5e-2 of max|out| elementwise."""
    from vcg_hip import ops
    from vcg_hip.build import build_two_stream
    from vcg_hip.trunk import ResNetTrunk, _tsm_info
    li, bi, H, Cin = blk_at
    T, N = 4, 12
    model = build_two_stream(clip_frame_num=T, seed=123, device=DEV, precision="bf16", dropout=0.0).eval()
    net = model.vision_model
    blk = getattr(net, f"layer{li}")[bi]
    g = torch.Generator().manual_seed(100 * li + bi)
    bns = [blk.bn1, blk.bn2, blk.bn3] + ([blk.downsample[1]] if blk.downsample is not None else [])
    with torch.no_grad():
        for bn in bns:
            C = bn.num_features
            bn.running_mean.copy_(torch.randn(C, generator=g) * 0.3)
            bn.running_var.copy_(torch.rand(C, generator=g) * 1.5 + 0.5)
            bn.weight.copy_(torch.rand(C, generator=g) + 0.5)
            bn.bias.copy_(torch.randn(C, generator=g) * 0.2)
    model.native_flat().refresh_shadow(force=True)
    x = torch.randn((N, H, H, Cin), generator=g).clamp_min(0).to(torch.bfloat16).to(DEV)
    trunk = ResNetTrunk(net, torch.bfloat16)
    trunk._fold_gen = object()
    conv1, T_, fold = _tsm_info(blk.conv1, Cin)
    with torch.no_grad():
        out_f = trunk._block_fwd_folded(blk, x, conv1, T_, fold, N, H, H)[0]
        ResNetTrunk.fold_eval = False
        try:
            out_u = trunk._block_fwd(blk, x, N, H, H, need_grad=False)[0]
        finally:
            ResNetTrunk.fold_eval = True
    torch.cuda.synchronize()
    a, b = out_f.double().cpu(), out_u.double().cpu()
    rel = ((a - b).norm() / b.norm()).item()
    err = (a - b).abs().max().item() / b.abs().max().item()
    print(f"layer{li}.{bi}: folded vs unfolded rel {rel:.2e}, max {err:.2e}")
    assert rel < 2e-2 and err < 5e-2


def test_folded_trunk_cache_and_whole_trunk():
    """The whole bf16 scoring trunk, folded vs unfolded, with running statistics calibrated on the same inputs (one
    batch-statistics forward with momentum 1). The random-init trunk amplifies bf16-sized perturbations ~25x: on the
    CPU oracle in fp64, multiplying the input frames by (1 + 4e-3 noise) alone moves these vision embeddings by 11 %
    (rel. Frobenius; fp32 vs fp64: 1.7e-5). The two bf16 paths differ by ~15 %, as each differs from fp32
    (test_gpu_bf16_train.py), so the per-block test above is the tight check. Here: within 0.25, logits within 5e-2, and the fold cache -- a second forward with the
    same state is bit-identical, a changed running statistic invalidates it."""
    from vcg_hip import synth
    from vcg_hip.build import build_two_stream
    from vcg_hip.trunk import ResNetTrunk
    T = 4
    model = build_two_stream(clip_frame_num=T, seed=123, device=DEV, precision="bf16", dropout=0.0)
    frames, ids, mask, _ = synth.clip_batch(4, T, 112, 112, 32, seed=11, device=DEV)
    for m in model.modules():
        if isinstance(m, torch.nn.BatchNorm2d):
            m.momentum = 1.0
    model.train()
    with torch.no_grad():
        model(frames, ids, mask)
    model.eval()
    outs = {}
    for fold in (True, False):
        ResNetTrunk.fold_eval = fold
        try:
            with torch.no_grad():
                logits, prob, vis, lang = model(frames, ids, mask, return_emb=True)
            torch.cuda.synchronize()
        finally:
            ResNetTrunk.fold_eval = True
        outs[fold] = (logits.float().cpu(), vis.float().cpu())
    (lf, vf), (lu, vu) = outs[True], outs[False]
    rel = ((vf - vu).norm() / vu.norm()).item()
    print(f"folded vs unfolded bf16 vision embeddings: rel Frobenius {rel:.3e}, max |dlogit| "
          f"{(lf - lu).abs().max().item():.3e}")
    assert rel < 0.25
    assert (lf - lu).abs().max().item() < 5e-2
    with torch.no_grad():
        l2, _, v2, _ = model(frames, ids, mask, return_emb=True)
    assert torch.equal(l2.float().cpu(), lf) and torch.equal(v2.float().cpu(), vf)
    bn = model.vision_model.layer4[2].bn3
    with torch.no_grad():
        bn.running_mean.add_(0.5)
        l3, _, _, _ = model(frames, ids, mask, return_emb=True)
    assert not torch.equal(l3.float().cpu(), lf)
