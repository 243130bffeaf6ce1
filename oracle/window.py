"""CPU fp32 restatement of StackedVideoChapterAttention, eval mode (TEST INFRASTRUCTURE ONLY — see
oracle/__init__.py). Pinned by tests/golden/window_attn.npz, produced by the reference module itself
(tools/oracle/make_golden_window.py).

`p` is a {state-dict name: tensor} dict with the reference's names relative to the module
(layers.{l}.attention.query.weight, ..., final_layer_norm.*, classifier.{0..16}.*).
"""
import math

import torch
import torch.nn.functional as F


def _lin(p, name, x):
    return F.linear(x, p[name + ".weight"], p[name + ".bias"])


def _ln(p, name, x):
    return F.layer_norm(x, (x.shape[-1],), p[name + ".weight"], p[name + ".bias"], 1e-5)


def window_attention(p, pre, x, nh):
    """VideoChapterWindowAttention.forward (stacked_window_self_attention.py:58-95), dropout inactive."""
    B, S, H = x.shape
    mid = S // 2
    pos = ((torch.arange(S) - mid).float() / (mid + 1e-6)).unsqueeze(-1)  # :48-52
    x = x + _lin(p, pre + "position_encoding", pos)                        # :69-72
    hd = H // nh

    def heads(t):
        return t.view(B, S, nh, hd).permute(0, 2, 1, 3)

    q, k, v = (heads(_lin(p, pre + n, x)) for n in ("query", "key", "value"))
    sc = q @ k.transpose(-1, -2) / math.sqrt(hd) + p[pre + "window_pos_bias"][:, :, :, :S]  # :79-83
    ctx = (F.softmax(sc, dim=-1) @ v).permute(0, 2, 1, 3).reshape(B, S, H)
    return _lin(p, pre + "out_proj", ctx)


def stacked_window_attention(p, emb, nh=16, n_layers=6):
    """StackedVideoChapterAttention.forward (:200-223): 6 pre-LN blocks (:131-145), final LN, middle clip,
    classifier (Linear LN GELU) x4 + Linear (:170-196), softmax. Returns logits, probs."""
    x = emb
    for l in range(n_layers):
        pre = f"layers.{l}."
        x = window_attention(p, pre + "attention.", _ln(p, pre + "attention_norm", x), nh) + x
        h = _ln(p, pre + "ffn_norm", x)
        for i in (0, 3, 6):
            h = F.gelu(_lin(p, pre + f"ffn.{i}", h))
        x = _lin(p, pre + "ffn.9", h) + x
    x = _ln(p, "final_layer_norm", x)[:, x.shape[1] // 2]
    for c in (0, 4, 8, 12):
        x = F.gelu(_ln(p, f"classifier.{c + 1}", _lin(p, f"classifier.{c}", x)))
    logits = _lin(p, "classifier.16", x)
    return logits, F.softmax(logits, dim=-1)


def _chain(p, pre, x, n_lin, final_relu=False):
    """Linear(pre.0) LN(pre.1) ReLU Dropout Linear(pre.4) ... Linear(pre.{4(n_lin-1)}) (eval)."""
    for j in range(n_lin):
        x = _lin(p, f"{pre}.{4 * j}", x)
        if j < n_lin - 1:
            x = F.relu(_ln(p, f"{pre}.{4 * j + 1}", x))
    return F.relu(x) if final_relu else x


def cross_attention(p, pre, lang, vis, nh=16):
    """CrossAttention.forward (two_stream_window.py:60-91), dropout inactive. lang [B, H], vis [B, T, H]."""
    B, T, H = vis.shape
    hd = H // nh
    lang = _ln(p, pre + "lang_norm", lang)
    vis = _ln(p, pre + "vision_norm", vis)
    pos = (torch.arange(T).float() / (T - 1)).unsqueeze(-1)  # :55-58
    vis = vis + _lin(p, pre + "frame_pos_encoding", pos)
    q = _lin(p, pre + "query_proj", lang).view(B, 1, nh, hd).transpose(1, 2)
    k = _lin(p, pre + "key_proj", vis).view(B, T, nh, hd).transpose(1, 2)
    v = _lin(p, pre + "value_proj", vis).view(B, T, nh, hd).transpose(1, 2)
    a = F.softmax(q @ k.transpose(-2, -1) / math.sqrt(hd), dim=-1)
    ctx = (a @ v).transpose(1, 2).reshape(B, H)
    return _lin(p, pre + "out_proj", ctx)


def chapter_head_mlp_window(p, lang_emb, vision_emb, i, prefix="fusion_head.", head_type="mlp"):
    """Window ChapterHead.forward (two_stream_window.py:251-288) for clip index i, head_type "mlp" or
    "cross_attn"."""
    B, T, _ = vision_emb.shape
    lang_out = _chain(p, f"{prefix}lang_proj_heads.{i}", lang_emb, 2, final_relu=True)
    vis_out = _chain(p, f"{prefix}vision_proj_heads.{i}", vision_emb.reshape(B * T, -1), 3, final_relu=True)
    if head_type == "cross_attn":
        return cross_attention(p, f"{prefix}head.", lang_out, vis_out.view(B, T, -1))
    if head_type == "self_attn":  # :280-282 (SelfAttention of two_stream_window.py:93-131, token 0 -> proj)
        x = torch.cat([vis_out.view(B, T, -1), lang_out.unsqueeze(1)], 1)
        C, nh = x.shape[-1], 4
        hs = C // nh

        def heads(name):
            return _lin(p, f"{prefix}head.{name}", x).view(B, T + 1, nh, hs).transpose(1, 2)
        k, q, v = heads("key"), heads("query"), heads("value")
        att = F.softmax((q @ k.transpose(-2, -1)) * (1.0 / math.sqrt(hs)), dim=-1)
        y = (att @ v).transpose(1, 2).reshape(B, T + 1, C)
        return _lin(p, f"{prefix}head.proj", y[:, 0])
    if head_type == "bilinear":  # :271-273
        w, b = p[f"{prefix}bilinear_layers.{i}.weight"], p[f"{prefix}bilinear_layers.{i}.bias"]
        fusion = F.bilinear(lang_out, vis_out.reshape(B, -1), w, b)
        x = F.relu(_ln(p, f"{prefix}head.{i}.0", fusion))
        x = F.relu(_ln(p, f"{prefix}head.{i}.4", _lin(p, f"{prefix}head.{i}.3", x)))
        return _lin(p, f"{prefix}head.{i}.7", x)
    if head_type == "multiplication":  # :275-279
        e = F.relu(_ln(p, f"{prefix}lang_expand_layers.{i}.1", _lin(p, f"{prefix}lang_expand_layers.{i}.0", lang_out)))
        e = F.relu(_ln(p, f"{prefix}lang_expand_layers.{i}.5", _lin(p, f"{prefix}lang_expand_layers.{i}.4", e)))
        return _chain(p, f"{prefix}head.{i}", vis_out.reshape(B, -1) * e, 3)
    fusion = torch.cat([vis_out.view(B, T, -1), lang_out.unsqueeze(1)], 1).reshape(B, -1)
    return _chain(p, f"{prefix}head.{i}", fusion, 3)


def two_stream_window(p, img_clips, ids, mask, bn_mode="running", nh=16, head_type="mlp"):
    """Window TwoStream.forward (two_stream_window.py:391-444): per clip BERT pooler + TSM-ResNet-50 + window
    ChapterHead, then StackedVideoChapterAttention. img_clips [B, n, T, 3, H, W], ids / mask [B, n, L]."""
    from .model import bert, resnet50_tsm
    B, n, T = img_clips.shape[:3]
    embs = []
    for i in range(n):
        lang_emb, _ = bert(p, ids[:, i], mask[:, i])
        vis = resnet50_tsm(p, img_clips[:, i].reshape(B * T, *img_clips.shape[3:]), T, bn_mode).view(B, T, -1)
        embs.append(chapter_head_mlp_window(p, lang_emb, vis, i, head_type=head_type))
    wp = {k[len("window_attn."):]: v for k, v in p.items() if k.startswith("window_attn.")}
    return stacked_window_attention(wp, torch.stack(embs, 1), nh=nh)
