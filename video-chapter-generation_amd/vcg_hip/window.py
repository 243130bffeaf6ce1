"""Window transformer (StackedVideoChapterAttention, reference model/fusion/stacked_window_self_attention.py:150-223)
on libvcg_hip: one launch of window_attn.hip per batch of windows (inference).

pack_window_weights() lays the module's f32 parameters out as window_attn.hip reads them (Linear weights
transposed to [in][out] so a workgroup reads one weight row per k-step as consecutive words):
  per layer l (6):  attention_norm g, b | query|key|value W^T [H][3H], bias [3H] | out_proj W^T [H][H], b |
                    position_encoding w [H] (Linear(1, H) weight column), b | window_pos_bias [nh][P] |
                    ffn_norm g, b | ffn.0 W^T [H][2H], b | ffn.3 W^T [2H][4H], b | ffn.6 W^T [4H][2H], b |
                    ffn.9 W^T [2H][H], b
  final_layer_norm g, b
  classifier c in (0, 4, 8, 12): W^T, b, then its LayerNorm (c + 1) g, b ; classifier.16 W^T [H/4][2], b
"""
import torch

from . import _lib
from .ops import P, _chk, stream


def _t(lin):
    return lin.weight.detach().t().contiguous().reshape(-1)


def pack_window_weights(m):
    """Flat f32 device buffer of a StackedVideoChapterAttention's parameters (layout above)."""
    parts = []
    for layer in m.layers:
        at = layer.attention
        parts += [layer.attention_norm.weight, layer.attention_norm.bias]
        parts.append(torch.cat([at.query.weight, at.key.weight, at.value.weight], 0).detach().t().contiguous()
                     .reshape(-1))
        parts += [torch.cat([at.query.bias, at.key.bias, at.value.bias]), _t(at.out_proj), at.out_proj.bias,
                  at.position_encoding.weight.reshape(-1), at.position_encoding.bias,
                  at.window_pos_bias.reshape(-1), layer.ffn_norm.weight, layer.ffn_norm.bias]
        for i in (0, 3, 6, 9):
            parts += [_t(layer.ffn[i]), layer.ffn[i].bias]
    parts += [m.final_layer_norm.weight, m.final_layer_norm.bias]
    for c in (0, 4, 8, 12):
        parts += [_t(m.classifier[c]), m.classifier[c].bias, m.classifier[c + 1].weight, m.classifier[c + 1].bias]
    parts += [_t(m.classifier[16]), m.classifier[16].bias]
    return torch.cat([p.detach().reshape(-1).float() for p in parts]).contiguous()


def window_attn_fwd(emb, weights, H, nh, P_len):
    """emb [B, S, H] f32 (GPU) -> logits, prob [B, 2] f32."""
    _chk(emb, torch.float32, "fusion_emb")
    _chk(weights, torch.float32, "packed window weights")
    B, S, Hd = emb.shape
    if Hd != H:
        raise RuntimeError(f"fusion_emb hidden size {Hd} != {H}")
    need = _lib.query("vcg_window_attn_weight_floats", H, nh, P_len)
    if weights.numel() != need:
        raise RuntimeError(f"packed window weights have {weights.numel()} floats, expected {need}")
    logits = torch.empty((B, 2), dtype=torch.float32, device=emb.device)
    prob = torch.empty((B, 2), dtype=torch.float32, device=emb.device)
    _lib.call("vcg_window_attn_fwd", P(emb), P(weights), weights.numel(), P(logits), P(prob), B, S, H, nh, P_len,
              stream())
    return logits, prob


def ln_act(x, ln, act):
    """act(LayerNorm(x)) for x [rows, D] f32 with an nn.LayerNorm's parameters (act: ops.ACT_*)."""
    _chk(x, torch.float32, "LayerNorm input")
    D = x.shape[-1]
    out = torch.empty_like(x)
    _lib.call("vcg_ln_act_fwd", P(x), P(ln.weight), P(ln.bias), P(out), x.numel() // D, D, float(ln.eps), int(act),
              stream())
    return out


def linear(x, lin, act=0):
    """act(x W^T + b) on the fp32 GEMM path (x [rows, in] f32)."""
    from .ops import gemm
    _chk(x, torch.float32, "Linear input")
    M, K = x.shape
    N = lin.weight.shape[0]
    return gemm(x, lin.weight, M, N, K, K, K, bias=lin.bias, act=act)


def mlp_chain(x, seq):
    """Run an nn.Sequential of Linear / LayerNorm / ReLU / GELU / Dropout (eval) natively: Linear + activation
    fuse into the GEMM epilogue, LayerNorm + activation into one row kernel."""
    from .ops import ACT_GELU, ACT_RELU
    mods = [m for m in seq if not isinstance(m, torch.nn.Dropout)]
    i = 0
    while i < len(mods):
        m = mods[i]
        nxt = mods[i + 1] if i + 1 < len(mods) else None
        act = ACT_RELU if isinstance(nxt, torch.nn.ReLU) else ACT_GELU if isinstance(nxt, torch.nn.GELU) else 0
        if isinstance(m, torch.nn.Linear):
            x = linear(x, m, act)
        elif isinstance(m, torch.nn.LayerNorm):
            x = ln_act(x, m, act)
        else:
            raise RuntimeError(f"mlp_chain: unsupported module {type(m).__name__}")
        i += 2 if act else 1
    return x


def pack_cross_attn_weights(ca):
    """Flat f32 buffer of a CrossAttention's parameters as cross_attn_fwd_kernel reads them: lang_norm g, b |
    vision_norm g, b | frame_pos_encoding w [H], b | query W^T [H][H], b | key|value W^T [H][2H], b [2H] |
    out_proj W^T [H][H], b."""
    parts = [ca.lang_norm.weight, ca.lang_norm.bias, ca.vision_norm.weight, ca.vision_norm.bias,
             ca.frame_pos_encoding.weight.reshape(-1), ca.frame_pos_encoding.bias, _t(ca.query_proj),
             ca.query_proj.bias,
             torch.cat([ca.key_proj.weight, ca.value_proj.weight], 0).detach().t().contiguous().reshape(-1),
             torch.cat([ca.key_proj.bias, ca.value_proj.bias]), _t(ca.out_proj), ca.out_proj.bias]
    return torch.cat([p.detach().reshape(-1).float() for p in parts]).contiguous()


def cross_attn_fwd(lang, vis, weights, H, nh):
    """lang [B, H], vis [B, T, H] f32 (GPU) -> [B, H] (two_stream_window.py CrossAttention.forward, eval)."""
    _chk(lang, torch.float32, "lang_out")
    _chk(vis, torch.float32, "vision_out")
    _chk(weights, torch.float32, "packed cross-attention weights")
    B, T, Hd = vis.shape
    if Hd != H or lang.shape != (B, H):
        raise RuntimeError(f"cross attention shapes: lang {tuple(lang.shape)}, vision {tuple(vis.shape)}, hidden {H}")
    if weights.numel() != _lib.query("vcg_cross_attn_weight_floats", H):
        raise RuntimeError("packed cross-attention weights have the wrong size")
    out = torch.empty((B, H), dtype=torch.float32, device=vis.device)
    _lib.call("vcg_cross_attn_fwd", P(lang), P(vis), P(weights), weights.numel(), P(out), B, T, H, nh, stream())
    return out


def mul(a, b):
    """a * b elementwise (f32, same shape)."""
    _chk(a, torch.float32, "mul operand")
    _chk(b, torch.float32, "mul operand")
    if a.shape != b.shape:
        raise RuntimeError(f"mul shapes differ: {tuple(a.shape)} vs {tuple(b.shape)}")
    out = torch.empty_like(a)
    _lib.call("vcg_mul_fwd", P(a), P(b), P(out), a.numel(), stream())
    return out


def bilinear(x1, x2, bl):
    """nn.Bilinear(x1 [B, I], x2 [B, J]) natively: U = x2 A^T (A = weight viewed [O*I][J], fp32 GEMM), then
    out[b][o] = sum_i U[b][o*I + i] x1[b][i] + bias[o] (vcg_rowdot_fwd)."""
    from .ops import gemm
    _chk(x1, torch.float32, "bilinear input1")
    _chk(x2, torch.float32, "bilinear input2")
    O, I, J = bl.weight.shape
    B = x1.shape[0]
    U = gemm(x2, bl.weight.detach().reshape(O * I, J), B, O * I, J, J, J)
    out = torch.empty((B, O), dtype=torch.float32, device=x1.device)
    _lib.call("vcg_rowdot_fwd", P(U), P(x1), P(bl.bias), P(out), B, O, I, stream())
    return out
