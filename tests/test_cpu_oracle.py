"""CPU suite: pins the oracle (oracle/) against the reference's golden vectors, and checks the
host-side logic and the C-ABI library surface (no GPU compute)."""
import json
import os

import numpy as np
import pytest
import torch

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def _gold(name):
    return np.load(os.path.join(GOLD, name), allow_pickle=False)


@pytest.fixture(scope="module")
def c1_params():
    from vcg_hip.build import build_two_stream
    from vcg_hip import synth
    torch.set_num_threads(min(8, os.cpu_count() or 8))
    m = build_two_stream(clip_frame_num=4, seed=123, bn_stats=dict(_gold("bn_running_stats.npz")), dropout=0.0)
    return m


def test_synthetic_inputs_match_golden():
    from vcg_hip import synth
    g = _gold("c1_fwd.npz")
    frames, ids, mask, labels = synth.clip_batch(2, 4, 112, 112, 32, seed=123)
    assert np.array_equal(ids.numpy(), g["c1_ids"])
    assert np.array_equal(mask.numpy(), g["c1_mask"])
    assert np.array_equal(labels.numpy(), g["c1_labels"])
    cs = g["c1_frames_checksum"]
    assert abs(frames.double().sum().item() - cs[0]) < 1e-9 * cs[1]


def test_state_dict_names_match_reference(c1_params):
    g = _gold("c1_train.npz")
    ref = [str(s) for s in g["train_grad_norm_names"]]
    ours = [n for n, _ in c1_params.named_parameters()]
    assert sorted(ours) == sorted(ref)
    assert sum(p.numel() for p in c1_params.lang_model.parameters()) == 109482240
    keys = set(c1_params.state_dict().keys())
    assert "vision_model.layer1.0.conv1.net.weight" in keys
    assert "vision_model.layer4.2.bn3.num_batches_tracked" in keys


@pytest.mark.parametrize("mode", ["running", "batch"])
def test_oracle_c1_forward_matches_reference(c1_params, mode):
    from oracle import model as om
    from vcg_hip import synth
    g = _gold("c1_fwd.npz")
    p = dict(c1_params.state_dict())
    frames, ids, mask, _ = synth.clip_batch(2, 4, 112, 112, 32, seed=123)
    with torch.no_grad():
        lg, pr, ve, le = om.two_stream(p, frames, ids, mask, bn_mode=mode)
    assert np.abs(lg.numpy() - g[f"c1_logits_{mode}"]).max() < 1e-5
    assert np.abs(pr.numpy() - g[f"c1_prob_{mode}"]).max() < 1e-5
    assert np.abs(le.numpy() - g["c1_lang_emb"]).max() < 1e-5
    assert np.abs(ve.numpy() - g[f"c1_vision_emb_{mode}"]).max() < 1e-5


def test_oracle_c1_train_step_matches_reference(c1_params):
    from oracle import model as om
    from vcg_hip import synth
    g = _gold("c1_train.npz")
    sd = c1_params.state_dict()
    names = [n for n, _ in c1_params.named_parameters()]
    params = {n: sd[n].detach().clone().requires_grad_() for n in names}
    buffers = {n: sd[n].detach().clone() for n in sd if n not in params}
    frames, ids, mask, labels = synth.clip_batch(2, 4, 112, 112, 32, seed=123)
    grads = {}
    for n, t in params.items():
        t.register_hook(lambda gr, n=n: grads.__setitem__(n, gr.detach().clone()))
    loss, logits, total, opt = om.train_step(params, buffers, frames, ids, mask, labels, lr=float(g["train_lr"][0]))
    assert abs(loss.item() - g["train_loss"][0]) < 1e-5
    assert abs(total.item() - g["train_total_norm"][0]) < 1e-4 * g["train_total_norm"][0]
    for key in [k for k in g.files if k.startswith("train_grad::")]:
        n = key.split("::", 1)[1]
        idx = g[f"train_idx::{n}"]
        ref = g[key]
        ours = grads[n].reshape(-1)[idx].numpy()
        assert np.abs(ours - ref).max() <= 1e-4 * max(np.abs(ref).max(), 1e-12), n
    for key in [k for k in g.files if k.startswith("train_rm::")]:
        n = key.split("::", 1)[1]
        assert np.abs(buffers[n + ".running_mean"].numpy() - g[key]).max() < 1e-5


def test_tsm_oracle_bitexact():
    from oracle import model as om
    g = _gold("tsm_shift.npz")
    x = torch.from_numpy(g["tsm_x"]).requires_grad_()
    y = om.tsm_shift(x, 4, 8)
    assert np.array_equal(y.detach().numpy(), g["tsm_y"])
    (gx,) = torch.autograd.grad(y, x, torch.from_numpy(g["tsm_g"]))
    assert np.array_equal(gx.numpy(), g["tsm_gx"])


def test_eval_utils_known_answers():
    from eval_utils.eval_utils import calculate_pr, convert_clip_label2cut_point
    with open(os.path.join(GOLD, "eval_utils.json")) as f:
        g = json.load(f)
    assert convert_clip_label2cut_point([1, 0, 0, 0, 1, 1, 0, 0, 1, 1, 1, 1, 1, 0, 1, 0, 0, 0, 0, 1, 1], 16, 2) == \
        [8, 26, 48, 64]
    for c in g["convert_clip_label2cut_point"]:
        assert convert_clip_label2cut_point(c["labels"], c["T"], c["off"]) == c["cut_points"]
    for c in g["calculate_pr"]:
        ours = calculate_pr(c["gt"], c["pred"])
        assert len(ours) == 6
        for a, b in zip(ours, c["pr"]):
            assert (a is None and b is None) or abs(a - b) < 1e-12


def test_optimizer_groups_match_reference_rule(c1_params):
    from vcg_hip.optim import param_groups
    from oracle.model import param_groups as oracle_groups
    ours = param_groups(c1_params, 0.01)
    ref = oracle_groups(list(c1_params.named_parameters()), 0.01)
    for a, b in zip(ours, ref):
        assert a["weight_decay"] == b["weight_decay"]
        assert {id(t) for t in a["params"]} == {id(t) for t in b["params"]}


def test_c_abi_library_exports_every_header_symbol():
    from vcg_hip import _lib
    protos = _lib.parse_header()
    assert len(protos) > 40
    lib = _lib.lib()  # binds every prototype; AttributeError if one is missing
    for name in protos:
        assert hasattr(lib, name)
    assert lib.vcg_version() == 1


def test_stem_bwd_fused_size_guard():
    """vcg_stem_bwd_fused addresses its operands with 32-bit buffer offsets: the host predicate admits the bench
    shapes and refuses a conv output of 4 GB or more (y = N x 112 x 112 x 64 bf16: >= 2675 frames), where the trunk
    runs the apply pass + weight gradient instead (host code only, no GPU)."""
    from vcg_hip import ops
    assert ops.stem_bwd_fused_fits(64 * 16, 112, 112)  # the C3 batch: 1024 frames, y 1.64 GB
    lim = 0xFFFFFF00
    n_max = (lim - 1) // (112 * 112 * 128)
    assert ops.stem_bwd_fused_fits(n_max, 112, 112)
    assert not ops.stem_bwd_fused_fits(n_max + 1, 112, 112)
    assert not ops.stem_bwd_fused_fits(168 * 16, 112, 112)
    assert not ops.stem_bwd_fused_fits(0, 112, 112)


def test_no_cpu_fallback():
    """The product path refuses CPU tensors loudly."""
    from vcg_hip import ops
    with pytest.raises(RuntimeError):
        ops.tsm_shift(torch.zeros(8, 64, 2, 2), 4, 8)


def _head_params(g):
    """The reference ChapterHead(attn) parameters of head_attn.npz, regenerated by name (vcg_hip/synth.py)."""
    from model.fusion.two_stream import ChapterHead
    from vcg_hip import synth
    h = ChapterHead(96, 160, 4, 128, 2, head_type="attn")
    synth.init_params(h, 123, prefix="fusion_head.")
    return {"fusion_head." + n: p.detach().clone().requires_grad_() for n, p in h.named_parameters()}


def test_oracle_attn_head_matches_reference():
    """oracle.chapter_head_attn against the reference SelfAttention head (two_stream.py:8-48): logits and the
    gradients of sum(logits * R) w.r.t. the inputs and every head parameter."""
    from oracle import model as om
    g = _gold("head_attn.npz")
    p = _head_params(g)
    lang = torch.from_numpy(g["head_lang"]).requires_grad_()
    vis = torch.from_numpy(g["head_vis"]).requires_grad_()
    lg = om.chapter_head_attn(p, lang, vis)
    assert np.abs(lg.detach().numpy() - g["head_logits"]).max() < 1e-5
    (lg * torch.from_numpy(g["head_R"])).sum().backward()
    assert np.abs(lang.grad.numpy() - g["head_dlang"]).max() < 1e-5
    assert np.abs(vis.grad.numpy() - g["head_dvis"]).max() < 1e-5
    for k in [k for k in g.files if k.startswith("head_grad::")]:
        n = "fusion_head." + k.split("::", 1)[1]
        ref = g[k]
        assert np.abs(p[n].grad.numpy() - ref).max() <= 1e-5 * (1 + np.abs(ref).max()), n


def test_oracle_c1_attn_forward_matches_reference():
    from oracle import model as om
    from vcg_hip.build import build_two_stream
    from vcg_hip import synth
    g = _gold("head_attn.npz")
    m = build_two_stream(clip_frame_num=4, seed=123, head_type="attn", bn_stats=dict(_gold("bn_running_stats.npz")),
                         dropout=0.0)
    frames, ids, mask, _ = synth.clip_batch(2, 4, 112, 112, 32, seed=123)
    with torch.no_grad():
        lg, pr, _, _ = om.two_stream(dict(m.state_dict()), frames, ids, mask, bn_mode="running", head_type="attn")
    assert np.abs(lg.numpy() - g["c1attn_logits_running"]).max() < 1e-5
    assert np.abs(pr.numpy() - g["c1attn_prob_running"]).max() < 1e-5


def _window_module(w):
    """The native StackedVideoChapterAttention (parameters only on CPU), initialised like the golden's
    reference module (vcg_hip/synth.py by state-dict name, prefix "window_attn.")."""
    from model.fusion.stacked_window_self_attention import StackedVideoChapterAttention
    from vcg_hip import synth
    cfg = type("Config", (), {"hidden_size": 128, "num_attention_heads": 16, "attention_probs_dropout_prob": 0.1,
                              "window_size": w})
    m = StackedVideoChapterAttention(cfg)
    synth.init_params(m, 123, prefix="window_attn.")
    return m.eval()


@pytest.mark.parametrize("case,w", [("w1", 1), ("w2", 2), ("short", 2)])
def test_oracle_window_attention_matches_reference(case, w):
    """oracle.window.stacked_window_attention against the reference StackedVideoChapterAttention
    (stacked_window_self_attention.py:148-223) on window_attn.npz; the native module's parameter names are
    the reference's (the golden's weights are regenerated by those names)."""
    from oracle import window as ow
    g = _gold("window_attn.npz")
    p = {n: t.detach() for n, t in _window_module(w).named_parameters()}
    lg, pr = ow.stacked_window_attention(p, torch.from_numpy(g[f"{case}_emb"]))
    assert np.abs(lg.numpy() - g[f"{case}_logits"]).max() < 1e-5
    assert np.abs(pr.numpy() - g[f"{case}_probs"]).max() < 1e-6


def test_window_weight_packing_layout():
    """pack_window_weights covers every parameter once, in the size the C-ABI expects
    (vcg_window_attn_weight_floats; a size query, no GPU compute)."""
    from vcg_hip import _lib
    from vcg_hip.window import pack_window_weights
    m = _window_module(2)
    flat = pack_window_weights(m)
    assert flat.numel() == sum(p.numel() for p in m.parameters())
    assert flat.numel() == _lib.query("vcg_window_attn_weight_floats", 128, 16, 5)
    # first layer: attention_norm gamma, beta, then [H][3H] = (query | key | value)^T
    at = m.layers[0].attention
    qkvT = flat[256:256 + 3 * 128 * 128].view(128, 384)
    assert torch.equal(qkvT[:, 128:256], at.key.weight.detach().t())


def _window_two_stream(w=1, T=4, device=None, head_type="mlp"):
    """The native window TwoStream (two_stream_window.py drop-in) built and initialised like the c1win golden."""
    import contextlib
    import io
    from model.fusion.two_stream_window import TwoStream
    from model.lang.bert_hugface import BertHugface
    from model.vision.resnet50_tsm import Resnet50TSM
    from vcg_hip import synth
    from vcg_hip.nn import BertConfig
    with contextlib.redirect_stdout(io.StringIO()):
        lang = BertHugface(pretrain_stage=False, config=BertConfig(output_attentions=True))
    vis = Resnet50TSM(segments_size=T, shift_div=8, pretrain_stage=False)
    m = TwoStream(lang.base_model, vis.base_model, lang.embed_size, vis.feature_dim, T, 128, w)
    m.build_chapter_head(output_size=2, head_type=head_type)
    if device is not None:
        m = m.to(device)
    synth.init_params(m, 123)
    synth.load_bn_stats(m, dict(_gold("bn_running_stats.npz")))
    return m.eval()


def _c1win_inputs(B=2, n=3, T=4, pad_first=False):
    from vcg_hip import synth
    frames, ids, mask, _ = synth.clip_batch(B * n, T, 112, 112, 32, seed=123)
    frames, ids, mask = frames.view(B, n, T, 3, 112, 112), ids.view(B, n, 32), mask.view(B, n, 32)
    if pad_first:  # zero padding clip (youtube_dataset.py:460-470)
        frames[:, 0] = 0
        ids[:, 0] = 0
        mask[:, 0] = 0
    return frames, ids, mask


WINDOW_HEADS = [("mlp", "c1win"), ("cross_attn", "c1xattn"), ("self_attn", "c1self_attn"),
                ("bilinear", "c1bilinear"), ("multiplication", "c1multiplication")]


@pytest.mark.parametrize("head_type,tag", WINDOW_HEADS)
def test_oracle_two_stream_window_matches_reference(head_type, tag):
    """oracle.window.two_stream_window against the reference window TwoStream (two_stream_window.py:291-444,
    head "mlp") at C1 shapes, running-stats eval; parameters by the native module's (= reference) names."""
    from oracle import window as ow
    torch.set_num_threads(min(8, os.cpu_count() or 8))
    g = _gold("window_attn.npz")
    m = _window_two_stream(head_type=head_type)
    p = {n: t.detach() for n, t in m.named_parameters()}
    p.update({n: b for n, b in m.named_buffers()})
    frames, ids, mask = _c1win_inputs()
    with torch.no_grad():
        lg, pr = ow.two_stream_window(p, frames, ids, mask, head_type=head_type)
    assert np.abs(lg.numpy() - g[f"{tag}_logits"]).max() < 1e-4
    assert np.abs(pr.numpy() - g[f"{tag}_prob"]).max() < 1e-4


def test_oracle_two_stream_window_padding_clip():
    """oracle.window.two_stream_window on the c1pad golden: clip 0 of each window is the zero padding clip
    (fully masked BERT input -> HF's uniform attention over all keys)."""
    from oracle import window as ow
    torch.set_num_threads(min(8, os.cpu_count() or 8))
    g = _gold("window_attn.npz")
    m = _window_two_stream()
    p = {n: t.detach() for n, t in m.named_parameters()}
    p.update({n: b for n, b in m.named_buffers()})
    with torch.no_grad():
        lg, _ = ow.two_stream_window(p, *_c1win_inputs(pad_first=True))
    assert np.abs(lg.numpy() - g["c1pad_logits"]).max() < 1e-4
