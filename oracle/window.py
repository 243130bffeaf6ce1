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
