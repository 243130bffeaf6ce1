"""End-to-end parity of the native TwoStream (libvcg_hip on MI355X) against the reference's own
outputs (tests/golden/*, produced by tools/oracle/make_golden.py running the reference modules).

Tolerances (written here, per north_star): fp32 parity mode — logits / prob within 1e-3 absolute;
embeddings within 1e-3 relative to their max; train-step gradients within 1e-3 of each tensor's
max |grad|. bf16 throughput mode is checked against the same fp32 goldens with a looser 5e-2 on
logits (bf16 activations through 53 convs + 12 layers; not a parity claim).

Train-step gradients: the fp32 reference itself deviates from exact (fp64) gradients by up to
1.9e-3 relative on vision BatchNorm parameter grads (ReLU / max-pool discontinuities and 8-frame
batch statistics amplify summation-order differences; measured with the oracle in fp64). Those
tensors therefore get 6e-3; every other gradient 2e-3 (and 99% of tensors must be within 2e-3).
"""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")
DEV = "cuda"


def _gold(name):
    return np.load(os.path.join(GOLD, name), allow_pickle=False)


@pytest.fixture(scope="module")
def stats():
    return dict(_gold("bn_running_stats.npz"))


def _model(T, stats, precision="fp32", dropout=0.0):
    from vcg_hip.build import build_two_stream
    return build_two_stream(clip_frame_num=T, seed=123, device=DEV, precision=precision, bn_stats=stats,
                            dropout=dropout)


def _batch_mode(model):
    # test_video_segment_point.py:116-122
    for m in model.modules():
        if isinstance(m, torch.nn.BatchNorm2d):
            m.track_running_stats = False
            m.running_mean = None
            m.running_var = None


def _inputs(B, T, HW, L):
    from vcg_hip import synth
    return synth.clip_batch(B, T, HW, HW, L, seed=123, device=DEV)


def _maxdiff(a, b):
    return float(np.abs(np.asarray(a, dtype=np.float64) - np.asarray(b, dtype=np.float64)).max())


def _check_fwd(model, g, tag, B, T, HW, L, tol_logits, mode):
    frames, ids, mask, labels = _inputs(B, T, HW, L)
    assert np.array_equal(ids.cpu().numpy(), g[f"{tag}_ids"])
    assert np.array_equal(mask.cpu().numpy(), g[f"{tag}_mask"])
    cs = g[f"{tag}_frames_checksum"]
    assert abs(frames.double().sum().item() - cs[0]) < 1e-6 * cs[1]
    with torch.no_grad():
        lg, pr, ve, le = model(frames, ids, mask, return_emb=True)
    torch.cuda.synchronize()
    d = _maxdiff(lg.cpu(), g[f"{tag}_logits_{mode}"])
    print(f"{tag} {mode} {model.precision}: max|dlogits| = {d:.3e}")
    assert d <= tol_logits, f"{tag} {mode} logits differ by {d}"
    assert _maxdiff(pr.cpu(), g[f"{tag}_prob_{mode}"]) <= tol_logits
    if model.precision == "fp32":
        lref = g[f"{tag}_lang_emb"]
        assert _maxdiff(le.cpu(), lref) <= 1e-3 * np.abs(lref).max()
        key = f"{tag}_vision_emb_{mode}"
        if key in g:
            vref = g[key]
            assert _maxdiff(ve.cpu(), vref) <= 1e-3 * np.abs(vref).max()
        else:
            vref = g[key + "_rows"]
            vv = ve.reshape(B * T, -1)[::37].cpu()
            assert _maxdiff(vv, vref) <= 1e-3 * np.abs(vref).max()


@pytest.mark.parametrize("mode", ["running", "batch"])
def test_c1_forward_fp32(stats, mode):
    g = _gold("c1_fwd.npz")
    model = _model(4, stats).eval()
    if mode == "batch":
        _batch_mode(model)
    _check_fwd(model, g, "c1", 2, 4, 112, 32, 1e-3, mode)


def test_c1_forward_bf16(stats):
    g = _gold("c1_fwd.npz")
    model = _model(4, stats, precision="bf16").eval()
    _check_fwd(model, g, "c1", 2, 4, 112, 32, 5e-2, "running")


def test_c1_train_step_fp32(stats):
    """One reference train step: BN train mode, dropout 0, CE, backward, clip_grad_norm_(1.0), AdamW."""
    from vcg_hip.functions import cross_entropy
    g = _gold("c1_train.npz")
    model = _model(4, stats).train()
    lr = float(g["train_lr"][0])

    class Cfg:
        weight_decay = 0.01
        learning_rate = lr
        betas = (0.9, 0.95)
    opt = model.configure_optimizers(Cfg)
    frames, ids, mask, labels = _inputs(2, 4, 112, 32)
    params = dict(model.named_parameters())
    before = {n: params[n].detach().clone() for n in params}
    logits, prob = model(frames, ids, mask)
    loss = cross_entropy(logits, labels)
    loss.backward()
    torch.cuda.synchronize()
    assert abs(loss.item() - g["train_loss"][0]) < 1e-4
    g64 = _gold("c1_train_fp64.npz")
    norms = {n: params[n].grad.double().norm().item() for n in params}
    names = [str(s) for s in g["train_grad_norm_names"]]
    ref_norms = dict(zip(names, g["train_grad_norms"]))
    exact_norms = dict(zip([str(s) for s in g64["norm_names"]], g64["norms"]))
    gmax = max(exact_norms.values())

    def tol(n):
        return 6e-3 if n.startswith("vision_model") and ("bn" in n or "downsample.1" in n) else 2e-3

    # (1) every gradient-tensor norm: as close to exact (fp64) as the fp32 reference, or within tol
    bad = []
    for n in names:
        ex = exact_norms[n] + 1e-7 * gmax
        e_ours = abs(norms[n] - exact_norms[n]) / ex
        e_ref = abs(ref_norms[n] - exact_norms[n]) / ex
        if e_ours > max(3 * e_ref, tol(n)):
            bad.append((n, e_ours, e_ref))
    assert not bad, f"{len(bad)} grad norms off, e.g. {bad[:5]}"
    # (2) sampled elements of tracked tensors, same criterion (relative to max|exact|)
    worst = []
    for key in [k for k in g.files if k.startswith("train_grad::")]:
        n = key.split("::", 1)[1]
        idx = g[f"train_idx::{n}"]
        gv = params[n].grad.reshape(-1)[torch.as_tensor(idx, device=DEV)].cpu().numpy()
        ex = g64[f"grad::{n}"]
        scale = max(np.abs(ex).max(), 1e-12)
        e_ours = _maxdiff(gv, ex) / scale
        e_ref = _maxdiff(g[key], ex) / scale
        worst.append((n, e_ours, e_ref))
        assert e_ours <= max(3 * e_ref, 1e-3), f"grad {n}: ours {e_ours:.2e} vs reference fp32 {e_ref:.2e}"
    print("grad error vs fp64 (ours, reference fp32):", [(n, f"{a:.1e}", f"{b:.1e}") for n, a, b in worst])
    total = opt.grad_norm().item()
    assert abs(total - g["train_total_norm"][0]) < 1e-3 * g["train_total_norm"][0]
    opt.clip_and_step(1.0)
    torch.cuda.synchronize()
    for key in [k for k in g.files if k.startswith("train_delta::")]:
        n = key.split("::", 1)[1]
        idx = torch.as_tensor(g[f"train_idx::{n}"], device=DEV)
        delta = (params[n].detach().reshape(-1)[idx] - before[n].reshape(-1)[idx]).cpu().numpy()
        ref = g[key]
        gref = np.abs(g64[f"grad::{n}"])
        # Adam's first step is ~lr*sign(g): compare where the exact gradient is well above the fp32 noise
        sel = gref > 0.05 * max(gref.max(), 1e-30)
        if sel.any():
            assert _maxdiff(delta[sel], ref[sel]) <= 0.05 * lr, f"delta {n}"
        ea = opt.state[params[n]]["exp_avg"].reshape(-1)[idx].cpu().numpy()
        eref = g[f"train_exp_avg::{n}"]
        # exp_avg = (1 - beta1) * clip_coef * grad: same criterion as the gradients
        ex = 0.1 * g64[f"grad::{n}"] * (1.0 / (g64["norms"] ** 2).sum() ** 0.5)
        scale = max(np.abs(ex).max(), 1e-12)
        e_ref = _maxdiff(eref, ex) / scale
        assert _maxdiff(ea, ex) / scale <= max(3 * e_ref, 2e-3), f"exp_avg {n}"
    bufs = dict(model.named_buffers())
    for key in [k for k in g.files if k.startswith("train_rm::")]:
        n = key.split("::", 1)[1]
        assert _maxdiff(bufs[n + ".running_mean"].cpu(), g[key]) <= 1e-4 * (1 + np.abs(g[key]).max())
        rv = g[f"train_rv::{n}"]
        assert _maxdiff(bufs[n + ".running_var"].cpu(), rv) <= 1e-4 * (1 + np.abs(rv).max())


@pytest.mark.skipif(not os.path.exists(os.path.join(GOLD, "c2_fwd.npz")), reason="c2 golden not generated")
@pytest.mark.parametrize("mode", ["running", "batch"])
def test_c2_forward_fp32(stats, mode):
    g = _gold("c2_fwd.npz")
    model = _model(16, stats).eval()
    if mode == "batch":
        _batch_mode(model)
    _check_fwd(model, g, "c2", 64, 16, 224, 128, 1e-3, mode)


def _head_module(dev):
    from model.fusion.two_stream import ChapterHead
    from vcg_hip import synth
    h = ChapterHead(96, 160, 4, 128, 2, head_type="attn").to(dev)
    synth.init_params(h, 123, prefix="fusion_head.")
    for p in h.parameters():
        p.grad = torch.zeros_like(p)
    return h


@pytest.mark.parametrize("precision", ["fp32", "bf16"])
def test_attn_head_kernels_vs_reference(precision):
    """vcg_head_attn_fwd / _bwd (+ the projection GEMMs as HeadEngine runs them) against the reference
    ChapterHead(attn) outputs and gradients (tests/golden/head_attn.npz). fp32: 1e-4 relative to each tensor's
    max; bf16 (activations and projection operands in bf16): 3e-2."""
    from vcg_hip import ops
    g = _gold("head_attn.npz")
    h = _head_module(DEV)
    dt = ops.torch_dtype(precision)
    B, T, hid = 3, 4, 128
    lang = torch.from_numpy(g["head_lang"]).to(DEV)
    vis = torch.from_numpy(g["head_vis"]).to(DEV).reshape(B * T, -1)
    lang_t, vis_t = lang.to(dt).contiguous(), vis.to(dt).contiguous()
    wv = h.vision_proj_head.weight.detach().to(dt).contiguous()
    wl = h.lang_proj_head.weight.detach().to(dt).contiguous()
    Vout = ops.gemm(vis_t, wv, B * T, hid, 160, 160, 160, act=ops.ACT_RELU)
    Lout = ops.gemm(lang_t, wl, B, hid, 96, 96, 96, act=ops.ACT_RELU)
    at = h.head
    logits, prob, saved = ops.head_attn_fwd(Vout, Lout, at.query, at.key, at.value, at.proj, B, T, hid, at.n_head)
    tol = 1e-4 if precision == "fp32" else 3e-2
    ref = g["head_logits"]
    assert _maxdiff(logits.cpu(), ref) <= tol * (1 + np.abs(ref).max())
    assert _maxdiff(prob.cpu(), torch.softmax(torch.from_numpy(ref), 1)) <= tol
    dlogits = torch.from_numpy(g["head_R"]).to(DEV)
    dV, dL = ops.head_attn_bwd(saved, at.query, at.key, at.value, at.proj, dlogits, Vout, Lout, B, T, hid, at.n_head)
    # the projections' gradients through the same GEMMs HeadEngine.backward uses
    ops.gemm_splitk(dV, vis_t, h.vision_proj_head.weight.grad, hid, 160, B * T, hid, 160, transA=True, transB=True)
    ops.gemm_splitk(dL, lang_t, h.lang_proj_head.weight.grad, hid, 96, B, hid, 96, transA=True, transB=True)
    dvis = ops.gemm(dV, wv, B * T, 160, hid, hid, 160, transB=True)
    dlang = ops.gemm(dL, wl, B, 96, hid, hid, 96, transB=True)
    torch.cuda.synchronize()
    for got, key in ((dvis.float().reshape(B, T, -1), "head_dvis"), (dlang.float(), "head_dlang")):
        r = g[key]
        assert _maxdiff(got.cpu(), r) <= tol * np.abs(r).max(), key
    for n, p in h.named_parameters():
        r = g[f"head_grad::{n}"]
        if precision == "fp32":
            d = _maxdiff(p.grad.cpu(), r)
            # key.bias: analytically zero (softmax is shift-invariant); the reference holds ~1e-9 rounding noise
            assert d <= tol * max(np.abs(r).max(), 1e-4), f"{n}: {d:.3e}"
        else:  # bf16 operands flip near-zero ReLU decisions of the 12-row batch: relative Frobenius error
            d = float(np.linalg.norm(p.grad.cpu().double().numpy() - r)) / max(float(np.linalg.norm(r)), 1e-4)
            assert d <= 5e-2, f"{n}: {d:.3e}"


def test_attn_head_dropout_regenerated_in_backward():
    """attn_drop in training: the backward regenerates the forward's mask from the seed. Checked through a
    directional derivative: <dlogits, d logits/dX . U> from vcg_head_attn_bwd equals the central difference of
    the forward along U (same seed, so the same mask)."""
    from vcg_hip import ops
    h = _head_module(DEV)
    at = h.head
    B, T, hid = 4, 4, 128
    gen = torch.Generator(device="cpu").manual_seed(3)
    Vout = (torch.rand(B * T, hid, generator=gen) + 0.1).to(DEV)
    Lout = (torch.rand(B, hid, generator=gen) + 0.1).to(DEV)
    U = torch.randn(B * T, hid, generator=gen).to(DEV)
    R = torch.randn(B, 2, generator=gen).to(DEV)
    seed, p = 12345, 0.3
    _, _, saved = ops.head_attn_fwd(Vout, Lout, at.query, at.key, at.value, at.proj, B, T, hid, at.n_head, p, seed)
    dV, _ = ops.head_attn_bwd(saved, at.query, at.key, at.value, at.proj, R, Vout, Lout, B, T, hid, at.n_head, p, seed,
                              relu_mask=False)
    eps = 1e-2
    lp, _, _ = ops.head_attn_fwd(Vout + eps * U, Lout, at.query, at.key, at.value, at.proj, B, T, hid, at.n_head, p,
                                 seed)
    lm, _, _ = ops.head_attn_fwd(Vout - eps * U, Lout, at.query, at.key, at.value, at.proj, B, T, hid, at.n_head, p,
                                 seed)
    fd = ((lp - lm) * R).sum().item() / (2 * eps)
    an = (dV * U).sum().item()
    assert abs(fd - an) <= 2e-3 * (1 + abs(an)), (fd, an)
    l0, _, _ = ops.head_attn_fwd(Vout, Lout, at.query, at.key, at.value, at.proj, B, T, hid, at.n_head, 0.0, seed)
    l1, _, _ = ops.head_attn_fwd(Vout, Lout, at.query, at.key, at.value, at.proj, B, T, hid, at.n_head, p, seed)
    assert _maxdiff(l0.cpu(), l1.cpu()) > 0  # the mask is applied


@pytest.mark.parametrize("precision", ["fp32", "bf16"])
def test_c1_attn_forward(stats, precision):
    """Full TwoStream C1 with head_type='attn' (running-stats eval) vs the reference golden."""
    from vcg_hip.build import build_two_stream
    g = _gold("head_attn.npz")
    model = build_two_stream(clip_frame_num=4, seed=123, device=DEV, precision=precision, bn_stats=stats,
                             dropout=0.0, head_type="attn").eval()
    frames, ids, mask, labels = _inputs(2, 4, 112, 32)
    with torch.no_grad():
        lg, pr = model(frames, ids, mask)
    tol = 1e-3 if precision == "fp32" else 5e-2
    assert _maxdiff(lg.cpu(), g["c1attn_logits_running"]) <= tol
    assert _maxdiff(pr.cpu(), g["c1attn_prob_running"]) <= tol


def test_c1_attn_train_step_runs(stats):
    """head_type='attn' through the whole native train step (fwd, bwd, clip + AdamW) in bf16 with dropout on:
    finite loss, every head parameter receives a gradient and moves."""
    from vcg_hip.build import build_two_stream
    from vcg_hip.functions import cross_entropy
    model = build_two_stream(clip_frame_num=4, seed=123, device=DEV, precision="bf16", bn_stats=stats,
                             dropout=0.1, head_type="attn").train()

    class Cfg:
        weight_decay = 0.01
        learning_rate = 1e-4
        betas = (0.9, 0.95)
    opt = model.configure_optimizers(Cfg)
    frames, ids, mask, labels = _inputs(2, 4, 112, 32)
    before = {n: p.detach().clone() for n, p in model.fusion_head.named_parameters()}
    opt.zero_grad()
    loss = cross_entropy(model(frames, ids, mask)[0], labels)
    loss.backward()
    for n, p in model.fusion_head.named_parameters():
        assert torch.isfinite(p.grad).all() and p.grad.abs().sum() > 0, n
    opt.clip_and_step(1.0)
    torch.cuda.synchronize()
    assert np.isfinite(loss.item())
    for n, p in model.fusion_head.named_parameters():
        assert not torch.equal(p.detach(), before[n]), n
