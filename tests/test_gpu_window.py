"""Window transformer StackedVideoChapterAttention (reference model/fusion/stacked_window_self_attention.py:148-223)
on libvcg_hip (window_attn.hip, inference): parity with the reference's own outputs (tests/golden/window_attn.npz,
tools/oracle/make_golden_window.py) and with the CPU oracle (oracle/window.py) at other shapes.

Tolerances (fp32 throughout, per north_star's 1e-3 on logits): golden cases 1e-4 absolute on logits and probs;
oracle cases (other hidden sizes / windows / batch 64) 1e-3 absolute.
"""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")
DEV = "cuda"


def _module(H, w, nh=16, seed=123):
    from model.fusion.stacked_window_self_attention import StackedVideoChapterAttention
    from vcg_hip import synth
    cfg = type("Config", (), {"hidden_size": H, "num_attention_heads": nh, "attention_probs_dropout_prob": 0.1,
                              "window_size": w})
    m = StackedVideoChapterAttention(cfg)
    synth.init_params(m, seed, prefix="window_attn.")
    return m.eval()


@pytest.mark.parametrize("case,w", [("w1", 1), ("w2", 2), ("short", 2)])
def test_window_attn_matches_reference_golden(case, w):
    g = np.load(os.path.join(GOLD, "window_attn.npz"), allow_pickle=False)
    m = _module(128, w).to(DEV)
    with torch.no_grad():
        lg, pr = m(torch.from_numpy(g[f"{case}_emb"]).to(DEV), None)
    torch.cuda.synchronize()
    assert np.abs(lg.cpu().numpy() - g[f"{case}_logits"]).max() < 1e-4
    assert np.abs(pr.cpu().numpy() - g[f"{case}_probs"]).max() < 1e-4


@pytest.mark.parametrize("H,w,nh,B", [(128, 2, 16, 64), (256, 3, 16, 8), (64, 7, 8, 5), (32, 0, 4, 3)])
def test_window_attn_matches_oracle(H, w, nh, B):
    from oracle import window as ow
    m = _module(H, w, nh, seed=7)
    gen = torch.Generator().manual_seed(H * 31 + w)
    emb = torch.randn(B, 2 * w + 1, H, generator=gen)
    p = {n: t.detach() for n, t in m.named_parameters()}
    ref_lg, ref_pr = ow.stacked_window_attention(p, emb, nh=nh)
    m = m.to(DEV)
    with torch.no_grad():
        lg, pr = m(emb.to(DEV))
    torch.cuda.synchronize()
    assert np.abs(lg.cpu().numpy() - ref_lg.numpy()).max() < 1e-3
    assert np.abs(pr.cpu().numpy() - ref_pr.numpy()).max() < 1e-3


@pytest.mark.parametrize("G", ["1", "2", "3", "5"])
def test_window_attn_windows_per_workgroup(G, monkeypatch):
    """Several windows per workgroup (VCG_WINDOW_G; the default picks G from the batch size): identical math per
    window, including a ragged last workgroup (B = 61)."""
    from oracle import window as ow
    monkeypatch.setenv("VCG_WINDOW_G", G)
    w = 1 if G == "5" else 2
    m = _module(128, w, seed=5)
    emb = torch.randn(61, 2 * w + 1, 128, generator=torch.Generator().manual_seed(3))
    ref_lg, _ = ow.stacked_window_attention({n: t.detach() for n, t in m.named_parameters()}, emb)
    m = m.to(DEV)
    with torch.no_grad():
        lg, _ = m(emb.to(DEV))
    torch.cuda.synchronize()
    assert np.abs(lg.cpu().numpy() - ref_lg.numpy()).max() < 1e-3


def test_window_attn_repacks_after_weight_update():
    m = _module(128, 1).to(DEV)
    emb = torch.randn(4, 3, 128, device=DEV)
    with torch.no_grad():
        a, _ = m(emb)
        m.classifier[16].bias.add_(1.0)  # in-place update bumps the parameter version
        b, _ = m(emb)
    torch.cuda.synchronize()
    assert torch.allclose(b - a, torch.ones_like(a), atol=1e-5)


def test_window_attn_rejects_bad_input():
    m = _module(128, 1).to(DEV)
    with pytest.raises(RuntimeError):
        m(torch.randn(2, 5, 128, device=DEV))  # more clips than 2w+1
    m.train()
    lg, pr = m(torch.randn(2, 3, 128, device=DEV))  # training: the native wtrain path (tests/test_gpu_window_train.py)
    torch.cuda.synchronize()
    assert torch.isfinite(lg).all() and lg.shape == (2, 2)


def test_ln_act_matches_torch():
    """vcg_ln_act_fwd (LayerNorm + ReLU / GELU row kernel) against torch fp32, rows of 96 / 1024 / 8 features."""
    import torch.nn.functional as F
    from vcg_hip.window import ln_act
    for rows, D, act in [(7, 96, 1), (300, 1024, 2), (5, 8, 0)]:
        ln = torch.nn.LayerNorm(D).to(DEV)
        with torch.no_grad():
            ln.weight.uniform_(0.5, 1.5)
            ln.bias.uniform_(-0.5, 0.5)
        x = torch.randn(rows, D, device=DEV) * 3 + 1
        ref = F.layer_norm(x, (D,), ln.weight, ln.bias, ln.eps)
        ref = F.relu(ref) if act == 1 else F.gelu(ref) if act == 2 else ref
        out = ln_act(x, ln, act)
        torch.cuda.synchronize()
        assert (out - ref).abs().max().item() < 1e-4


@pytest.mark.parametrize("T,H,nh,B", [(16, 128, 16, 64), (4, 128, 16, 3), (2, 64, 8, 5)])
def test_cross_attn_matches_oracle(T, H, nh, B):
    """vcg_cross_attn_fwd (window ChapterHead "cross_attn", two_stream_window.py:11-91) against the oracle."""
    from model.fusion.two_stream_window import CrossAttention
    from oracle import window as ow
    from vcg_hip import synth
    from vcg_hip.window import cross_attn_fwd, pack_cross_attn_weights
    ca = CrossAttention(H, nh)
    synth.init_params(ca, 9, prefix="fusion_head.head.")
    gen = torch.Generator().manual_seed(T * 7 + H)
    lang, vis = torch.rand(B, H, generator=gen), torch.rand(B, T, H, generator=gen)  # post-ReLU-like inputs
    ref = ow.cross_attention({n: t.detach() for n, t in ca.named_parameters()}, "", lang, vis, nh=nh)
    ca = ca.to(DEV)
    out = cross_attn_fwd(lang.to(DEV), vis.to(DEV), pack_cross_attn_weights(ca), H, nh)
    torch.cuda.synchronize()
    assert (out.cpu() - ref).abs().max().item() < 1e-4


@pytest.mark.parametrize("head_type,tag", [("mlp", "c1win"), ("cross_attn", "c1xattn"), ("self_attn", "c1self_attn"),
                                          ("bilinear", "c1bilinear"), ("multiplication", "c1multiplication")])
def test_two_stream_window_matches_reference_golden(head_type, tag):
    """The native window TwoStream (BERT + TSM-ResNet-50 engines per clip, window ChapterHead "mlp" on the fp32
    GEMM / LN kernels or the cross-attention kernel, window transformer kernel) against the reference's own output
    at C1 shapes (c1win / c1xattn, 3 clips
    of 4 x 112^2 + 32 tokens, batch 2, running-stats eval): logits / prob within 1e-3."""
    from test_cpu_oracle import _c1win_inputs, _window_two_stream
    g = np.load(os.path.join(GOLD, "window_attn.npz"), allow_pickle=False)
    m = _window_two_stream(device=DEV, head_type=head_type)
    frames, ids, mask = _c1win_inputs()
    with torch.no_grad():
        lg, pr = m(frames.to(DEV), ids.to(DEV), mask.to(DEV), None)
    torch.cuda.synchronize()
    assert np.abs(lg.cpu().numpy() - g[f"{tag}_logits"]).max() < 1e-3
    assert np.abs(pr.cpu().numpy() - g[f"{tag}_prob"]).max() < 1e-3


def test_two_stream_window_padding_clip_matches_reference_golden():
    """A window that runs off the start of the video: clip 0 is the reference's zero padding (frames, text ids and
    attention mask all 0, youtube_dataset.py:460-470) -- BERT sees a fully masked sequence there (c1pad golden)."""
    from test_cpu_oracle import _c1win_inputs, _window_two_stream
    g = np.load(os.path.join(GOLD, "window_attn.npz"), allow_pickle=False)
    m = _window_two_stream(device=DEV)
    frames, ids, mask = _c1win_inputs(pad_first=True)
    with torch.no_grad():
        lg, pr = m(frames.to(DEV), ids.to(DEV), mask.to(DEV), None)
    torch.cuda.synchronize()
    assert np.isfinite(lg.cpu().numpy()).all()
    assert np.abs(lg.cpu().numpy() - g["c1pad_logits"]).max() < 1e-3


def test_window_scoring_from_clip_embeddings_matches_forward():
    """TwoStream.forward_embeddings (each clip's BERT / trunk pass once, windows gathered from the per-clip
    embeddings, -1 = the zero padding clip) equals forward() on the materialised windows (C1 shapes, w = 1)."""
    from test_cpu_oracle import _window_two_stream
    from vcg_hip import synth
    m = _window_two_stream(device=DEV)
    N, T, L = 5, 4, 32
    frames, ids, mask, _ = synth.clip_batch(N, T, 112, 112, L, seed=77, device=DEV)
    win = torch.tensor([[-1, 0, 1], [0, 1, 2], [2, 3, 4], [3, 4, -1], [1, 3, 0]], device=DEV)
    zf = torch.zeros((1, T, 3, 112, 112), device=DEV)
    zi = torch.zeros((1, L), dtype=torch.long, device=DEV)
    with torch.no_grad():
        lang, vis = m.clip_embeddings(frames, ids, mask, chunk=2)
        pl, pv = m.clip_embeddings(zf, zi, zi)
        lg, pr = m.forward_embeddings(lang, vis, win, pl[0], pv[0])
        allf, alli, allm = torch.cat([frames, zf]), torch.cat([ids, zi]), torch.cat([mask, zi])
        sel = torch.where(win < 0, torch.full_like(win, N), win)
        lg_ref, _ = m(allf[sel], alli[sel], allm[sel], None)
    torch.cuda.synchronize()
    assert torch.isfinite(lg).all()
    assert (lg - lg_ref).abs().max().item() < 1e-4


def test_window_kernels_empty_batch():
    """B = 0 windows: the C-ABI returns at once and the wrappers give empty [0, 2] / [0, H] results."""
    from model.fusion.two_stream_window import CrossAttention
    from vcg_hip.window import cross_attn_fwd, pack_cross_attn_weights
    m = _module(128, 1).to(DEV)
    with torch.no_grad():
        lg, pr = m(torch.empty((0, 3, 128), device=DEV))
        ca = CrossAttention(128, 16).to(DEV)
        out = cross_attn_fwd(torch.empty((0, 128), device=DEV), torch.empty((0, 4, 128), device=DEV),
                             pack_cross_attn_weights(ca), 128, 16)
    torch.cuda.synchronize()
    assert lg.shape == (0, 2) and pr.shape == (0, 2) and out.shape == (0, 128)
