"""Training path of the window model on libvcg_hip: reference model/fusion/two_stream_window.py
(ChapterHead 134-288, CrossAttention 11-91, SelfAttention 93-131, TwoStream 291-444) and
stacked_window_self_attention.py (VideoChapterWindowAttention 6-95, VideoChapterBlock 98-145,
StackedVideoChapterAttention 148-223), as trained by train_video_segment_ddp.py:294-342.

Every op is a torch.autograd.Function whose forward AND backward are libvcg_hip kernels (fp32, as the reference
runs these heads): Linear -> vcg_gemm (bias / ReLU / residual in the epilogue; dX by vcg_gemm, dW by the split-K
GEMM, db by vcg_colsum); LayerNorm + activation + Dropout -> vcg_ln_act_drop_fwd / _bwd; activation + Dropout (+
residual) -> vcg_act_drop_*; the window / cross attention core -> vcg_mha_small_*; the SelfAttention head ->
vcg_head_attn_*; the elementwise product -> vcg_mul_*. Parameter gradients are ACCUMULATED by the kernels into the
parameters' .grad (views of the model's flat gradient buffer), so the Functions return no parameter gradients.
Dropout masks are regenerated in the backward from a per-call seed (counter hash): same masks, no mask tensors.
torch is used for memory (allocation, views, cat / slice copies) only.
"""
import math

import numpy as np
import torch

from . import _lib, ops
from .nn import new_seed
from .ops import P, stream

ACT_NONE, ACT_RELU, ACT_GELU = 0, 1, 2


def _grad(p):
    """p.grad (a flat-buffer view under NativeRoot), created as zeros if absent."""
    if p is None or not p.requires_grad:
        return None
    if p.grad is None:
        p.grad = torch.zeros_like(p)
    return p.grad


class CastF32Fn(torch.autograd.Function):
    """compute-dtype (bf16) encoder output -> f32 head input; the gradient goes back in the input's dtype."""

    @staticmethod
    def forward(ctx, x):
        ctx.dt = x.dtype
        return ops.cast_to_f32(x.contiguous())

    @staticmethod
    def backward(ctx, d):
        return ops.cast_from_f32(d.contiguous(), ctx.dt)


def _f32(x):
    return CastF32Fn.apply(x) if x.dtype != torch.float32 else x.contiguous()


def _drop_p(m):
    return float(m.p) if (m is not None and m.training) else 0.0


# ------------------------------------------------------------------------------------------------ Functions
class LinearFn(torch.autograd.Function):
    """y = act(x W^T + b + res) for x [M, K]; act none / ReLU (the ReLU mask is read back from y)."""

    @staticmethod
    def forward(ctx, x, lin, act, res):
        M, K = x.shape
        N = lin.weight.shape[0]
        ctx.small = (N % 4 != 0) or (K % 4 != 0)  # below the GEMM's 16-byte tiles (the 2-way classifiers)
        if ctx.small:
            y = torch.empty((M, N), dtype=torch.float32, device=x.device)
            _lib.call("vcg_linear_small_fwd", P(x), P(lin.weight), P(lin.bias), P(res), P(y), M, N, K, int(act),
                      stream())
        else:
            y = ops.gemm(x, lin.weight, M, N, K, K, K, bias=lin.bias, act=act, residual=res, ldr=N)
        ctx.lin, ctx.act = lin, act
        ctx.save_for_backward(x, y if act == ACT_RELU else None)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, y = ctx.saved_tensors
        lin, act = ctx.lin, ctx.act
        dy = dy.contiguous()
        M, K = x.shape
        N = lin.weight.shape[0]
        if act == ACT_RELU:
            g = torch.empty_like(dy)
            _lib.call("vcg_act_drop_bwd", P(dy), P(y), P(g), g.numel(), ACT_RELU, 0.0, 0, stream())
        else:
            g = dy
        if ctx.small:
            dx = torch.empty_like(x) if ctx.needs_input_grad[0] else None
            _lib.call("vcg_linear_small_bwd", P(g), P(x), P(lin.weight), P(dx), P(_grad(lin.weight)),
                      P(_grad(lin.bias)), M, N, K, stream())
            return dx, None, None, (g if ctx.needs_input_grad[3] else None)
        gw = _grad(lin.weight)
        if gw is not None:
            ops.gemm_splitk(g, x, gw, N, K, M, N, K, transA=True, transB=True)
        gb = _grad(lin.bias)
        if gb is not None:
            ops.colsum(g, N, M, N, gb, accumulate=True)
        dx = ops.gemm(g, lin.weight, M, K, N, N, K, transB=True) if ctx.needs_input_grad[0] else None
        return dx, None, None, (g if ctx.needs_input_grad[3] else None)


class BilinearFn(torch.autograd.Function):
    """nn.Bilinear(x1 [B, I], x2 [B, J]) -> [B, O] (the "bilinear" window ChapterHead, two_stream_window.py:187-191,
    269-273): U = x2 A^T (A = weight viewed [O*I][J]), y[b][o] = sum_i U[b][o*I + i] x1[b][i] + bias[o]
    (vcg_rowdot_fwd). Backward: dU = dy (x) x1 and dx1 = sum_o dy U (vcg_rowdot_bwd), dx2 = dU A (GEMM),
    dA += dU^T x2 (split-K GEMM), dbias += colsum(dy)."""

    @staticmethod
    def forward(ctx, x1, x2, bl):
        O, I, J = bl.weight.shape
        B = x1.shape[0]
        x1, x2 = x1.contiguous(), x2.contiguous()
        U = ops.gemm(x2, bl.weight.detach().reshape(O * I, J), B, O * I, J, J, J)
        y = torch.empty((B, O), dtype=torch.float32, device=x1.device)
        _lib.call("vcg_rowdot_fwd", P(U), P(x1), P(bl.bias), P(y), B, O, I, stream())
        ctx.bl = bl
        ctx.save_for_backward(x1, x2, U)
        return y

    @staticmethod
    def backward(ctx, dy):
        x1, x2, U = ctx.saved_tensors
        bl = ctx.bl
        O, I, J = bl.weight.shape
        B = x1.shape[0]
        dy = dy.contiguous()
        dU = torch.empty_like(U)
        dx1 = torch.empty_like(x1) if ctx.needs_input_grad[0] else None
        _lib.call("vcg_rowdot_bwd", P(U), P(x1), P(dy), P(dU), P(dx1), B, O, I, stream())
        gw = _grad(bl.weight)
        if gw is not None:
            ops.gemm_splitk(dU, x2, gw.view(O * I, J), O * I, J, B, O * I, J, transA=True, transB=True)
        gb = _grad(bl.bias)
        if gb is not None:
            ops.colsum(dy, O, B, O, gb, accumulate=True)
        dx2 = None
        if ctx.needs_input_grad[1]:
            dx2 = ops.gemm(dU, bl.weight.detach().reshape(O * I, J), B, J, O * I, O * I, J, transB=True)
        return dx1, dx2, None


class LNActDropFn(torch.autograd.Function):
    """Dropout(act(LayerNorm(x))) for x [rows, D]."""

    @staticmethod
    def forward(ctx, x, ln, act, p):
        rows, D = x.shape
        out = torch.empty_like(x)
        mean = torch.empty(rows, dtype=torch.float32, device=x.device)
        rstd = torch.empty_like(mean)
        seed = new_seed() if p > 0.0 else 0
        _lib.call("vcg_ln_act_drop_fwd", P(x), P(ln.weight), P(ln.bias), P(out), P(mean), P(rstd), rows, D,
                  float(ln.eps), int(act), float(p), seed, stream())
        ctx.ln, ctx.act, ctx.p, ctx.seed = ln, act, p, seed
        ctx.save_for_backward(x, mean, rstd)
        return out

    @staticmethod
    def backward(ctx, dout):
        x, mean, rstd = ctx.saved_tensors
        ln = ctx.ln
        rows, D = x.shape
        dx = torch.empty_like(x)
        w = ops.ws(_lib.query("vcg_ln_act_drop_bwd_ws_bytes", rows, D), x.device)
        _lib.call("vcg_ln_act_drop_bwd", P(dout.contiguous()), P(x), P(ln.weight), P(ln.bias), P(mean), P(rstd), P(dx),
                  P(_grad(ln.weight)), P(_grad(ln.bias)), P(w), w.numel() * 4, rows, D, int(ctx.act), float(ctx.p),
                  ctx.seed, stream())
        return dx, None, None, None


class ActDropFn(torch.autograd.Function):
    """Dropout(act(x)) (+ res), elementwise."""

    @staticmethod
    def forward(ctx, x, act, p, res):
        out = torch.empty_like(x)
        seed = new_seed() if p > 0.0 else 0
        _lib.call("vcg_act_drop_fwd", P(x), P(res), P(out), x.numel(), int(act), float(p), seed, stream())
        ctx.act, ctx.p, ctx.seed = act, p, seed
        ctx.save_for_backward(x)
        return out

    @staticmethod
    def backward(ctx, dout):
        (x,) = ctx.saved_tensors
        dout = dout.contiguous()
        dx = torch.empty_like(x)
        _lib.call("vcg_act_drop_bwd", P(dout), P(x), P(dx), x.numel(), int(ctx.act), float(ctx.p), ctx.seed, stream())
        return dx, None, None, (dout if ctx.needs_input_grad[3] else None)


class MulFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, a, b):
        out = torch.empty_like(a)
        _lib.call("vcg_mul_fwd", P(a), P(b), P(out), a.numel(), stream())
        ctx.save_for_backward(a, b)
        return out

    @staticmethod
    def backward(ctx, dout):
        a, b = ctx.saved_tensors
        da, db = torch.empty_like(a), torch.empty_like(b)
        _lib.call("vcg_mul_bwd", P(dout.contiguous()), P(a), P(b), P(da), P(db), a.numel(), stream())
        return da, db


class MHAFn(torch.autograd.Function):
    """Short-window multi-head attention core: q [B*Sq, H], k / v [B*Sk, H] -> ctx [B*Sq, H]; optional per-head key
    bias parameter [.., nh, .., Pb] (window_pos_bias)."""

    @staticmethod
    def forward(ctx, q, k, v, bias, B, Sq, Sk, nh, p):
        H = q.shape[1]
        dh = H // nh
        scale = 1.0 / math.sqrt(dh)
        out = torch.empty_like(q)
        probs = torch.empty(B * nh * Sq * Sk, dtype=torch.float32, device=q.device)
        Pb = bias.shape[-1] if bias is not None else 0
        seed = new_seed() if p > 0.0 else 0
        _lib.call("vcg_mha_small_fwd", P(q), H, P(k), H, P(v), H, P(bias), Pb, P(out), H, P(probs), B, Sq, Sk, nh, dh,
                  float(scale), float(p), seed, stream())
        ctx.bias, ctx.dims, ctx.seed = bias, (B, Sq, Sk, nh, dh, scale, p, Pb), seed
        ctx.save_for_backward(q, k, v, probs)
        return out

    @staticmethod
    def backward(ctx, dctx):
        q, k, v, probs = ctx.saved_tensors
        B, Sq, Sk, nh, dh, scale, p, Pb = ctx.dims
        H = q.shape[1]
        dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
        gb = _grad(ctx.bias) if ctx.bias is not None else None
        w = ops.ws(_lib.query("vcg_mha_small_bwd_ws_bytes", B, nh, max(Pb, 1)), q.device)
        _lib.call("vcg_mha_small_bwd", P(q), H, P(k), H, P(v), H, P(probs), P(dctx.contiguous()), H, P(dq), H, P(dk), H,
                  P(dv), H, P(gb), Pb, P(w), w.numel() * 4, B, Sq, Sk, nh, dh, float(scale), float(p), ctx.seed,
                  stream())
        return dq, dk, dv, None, None, None, None, None, None


class PosEncFn(torch.autograd.Function):
    """x + Linear(1, H)(pos) per token (pos: S position scalars, token r uses pos[r % S])."""

    @staticmethod
    def forward(ctx, x, lin, pos):
        rows, H = x.shape
        out = torch.empty_like(x)
        _lib.call("vcg_posenc_fwd", P(x), P(pos), P(lin.weight), P(lin.bias), P(out), rows, pos.numel(), H, stream())
        ctx.lin = lin
        ctx.save_for_backward(pos)
        ctx.shape = (rows, H)
        return out

    @staticmethod
    def backward(ctx, dout):
        (pos,) = ctx.saved_tensors
        rows, H = ctx.shape
        dout = dout.contiguous()
        _lib.call("vcg_posenc_bwd", P(dout), P(pos), P(_grad(ctx.lin.weight)), P(_grad(ctx.lin.bias)), rows,
                  pos.numel(), H, stream())
        return dout, None, None


class HeadAttnFn(torch.autograd.Function):
    """ChapterHead "self_attn" (two_stream_window.py:280-282): SelfAttention over cat([vision_out, lang_out]) ->
    proj of token 0, on the head_attn kernels (the inputs' ReLU masks are applied by their LinearFn)."""

    @staticmethod
    def forward(ctx, vis, lang, at, B, T, hid):
        p = _drop_p(at.attn_drop)
        seed = new_seed() if p > 0.0 else 0
        # resid_drop is declared but never applied by the reference (two_stream_window.py:108 vs :114-131), so it is
        # ignored here too at any p.
        out, _, saved = ops.head_attn_fwd(vis, lang, at.query, at.key, at.value, at.proj, B, T, hid, at.n_head, p, seed)
        ctx.at, ctx.dims, ctx.p, ctx.seed, ctx.saved_state = at, (B, T, hid), p, seed, saved
        ctx.save_for_backward(vis, lang)
        return out

    @staticmethod
    def backward(ctx, dout):
        vis, lang = ctx.saved_tensors
        at = ctx.at
        B, T, hid = ctx.dims
        for lin in (at.query, at.key, at.value, at.proj):
            _grad(lin.weight)
            _grad(lin.bias)
        dV, dL = ops.head_attn_bwd(ctx.saved_state, at.query, at.key, at.value, at.proj, dout.contiguous(), vis, lang,
                                   B, T, hid, at.n_head, ctx.p, ctx.seed, relu_mask=False)
        return dV, dL, None, None, None, None


def softmax_rows(logits):
    """prob = softmax(logits, 1) (reported; the loss comes from the cross-entropy kernels)."""
    with torch.no_grad():
        out = torch.empty_like(logits)
        _lib.call("vcg_softmax_rows", P(logits.contiguous()), P(out), logits.shape[0], logits.shape[1], stream())
    return out


# ------------------------------------------------------------------------------------------------ module walks
def linear(x, lin, act=ACT_NONE, res=None):
    return LinearFn.apply(x, lin, act, res)


def chain(x, seq, final_act=ACT_NONE, res=None):
    """Run an nn.Sequential of Linear / LayerNorm / ReLU / GELU / Dropout in training mode. Each Linear or
    LayerNorm takes the activation and Dropout that follow it: Linear + ReLU (no dropout) -> one GEMM epilogue,
    LayerNorm + act + Dropout -> one row kernel, act + Dropout after a Linear -> one elementwise kernel.
    `final_act` (F.relu applied to the sequence's output) joins the last module; `res` is added after it."""
    mods = list(seq)
    n, i = len(mods), 0
    while i < n:
        m = mods[i]
        j, act, drop = i + 1, ACT_NONE, None
        if j < n and isinstance(mods[j], (torch.nn.ReLU, torch.nn.GELU)):
            act = ACT_RELU if isinstance(mods[j], torch.nn.ReLU) else ACT_GELU
            j += 1
        if j < n and isinstance(mods[j], torch.nn.Dropout):
            drop = mods[j]
            j += 1
        last = j >= n
        if last and final_act != ACT_NONE:
            if act != ACT_NONE:
                raise RuntimeError("chain: final_act after an activation")
            act = final_act
        p = _drop_p(drop)
        r = res if last else None
        if isinstance(m, torch.nn.Linear):
            if p == 0.0 and act in (ACT_NONE, ACT_RELU):
                x = linear(x, m, act, r if act == ACT_NONE else None)
                if r is not None and act != ACT_NONE:
                    x = ActDropFn.apply(x, ACT_NONE, 0.0, r)
            else:
                x = ActDropFn.apply(linear(x, m), act, p, r)
        elif isinstance(m, torch.nn.LayerNorm):
            x = LNActDropFn.apply(x, m, act, p)
            if r is not None:
                x = ActDropFn.apply(x, ACT_NONE, 0.0, r)
        else:
            raise RuntimeError(f"chain: unsupported module {type(m).__name__}")
        i = j
    return x


def layer_norm(x, ln):
    return LNActDropFn.apply(x, ln, ACT_NONE, 0.0)


def _positions(values, device):
    return torch.from_numpy(np.asarray(values, dtype=np.float32)).to(device)


# ------------------------------------------------------------------------------------------------ ChapterHead
def cross_attention(ca, lang_out, vision_out, B, T):
    """CrossAttention.forward (two_stream_window.py:55-91): lang_out [B, H], vision_out [B*T, H] -> [B, H]."""
    H = ca.hidden_size
    ln_l = layer_norm(lang_out, ca.lang_norm)
    ln_v = layer_norm(vision_out, ca.vision_norm)
    # get_relative_positions :51-53, in fp32 as torch computes it
    pos = _positions(np.arange(T, dtype=np.float32) / np.float32(T - 1), vision_out.device)
    vis = PosEncFn.apply(ln_v, ca.frame_pos_encoding, pos)                   # vision_emb + position_emb
    q = linear(ln_l, ca.query_proj)
    k = linear(vis, ca.key_proj)
    v = linear(vis, ca.value_proj)
    ctx = MHAFn.apply(q, k, v, None, B, 1, T, ca.num_heads, _drop_p(ca.attention_dropout))
    out = linear(ctx, ca.out_proj)
    p = _drop_p(ca.output_dropout)
    return ActDropFn.apply(out, ACT_NONE, p, None) if p > 0.0 else out


def chapter_head(hd, lang_emb, vision_emb, i):
    """ChapterHead.forward(lang_emb [B, Dl], vision_emb [B, T, Dv], window_idx=i) in training (:251-288)."""
    B, T, h = lang_emb.shape[0], hd.segment_size, hd.hidden_size
    lang_out = chain(_f32(lang_emb), hd.lang_proj_heads[i], final_act=ACT_RELU)                    # :262-263
    vision_out = chain(_f32(vision_emb.reshape(B * T, -1)), hd.vision_proj_heads[i], final_act=ACT_RELU)  # :265-267
    if hd.head_type == "mlp":                                                                      # :269-272
        fusion = torch.cat([vision_out.view(B, T, h), lang_out.view(B, 1, h)], 1).view(B, (T + 1) * h)
        return chain(fusion, hd.head[i])
    if hd.head_type == "multiplication":                                                           # :275-279
        expanded = chain(lang_out, hd.lang_expand_layers[i])
        return chain(MulFn.apply(vision_out.view(B, T * h), expanded.view(B, T * h)), hd.head[i])
    if hd.head_type == "self_attn":                                                                # :280-282
        return HeadAttnFn.apply(vision_out, lang_out, hd.head, B, T, h)
    if hd.head_type == "cross_attn":                                                               # :284-286
        return cross_attention(hd.head, lang_out, vision_out, B, T)
    if hd.head_type == "bilinear":                                                                 # :269-273
        return chain(BilinearFn.apply(lang_out, vision_out.view(B, T * h), hd.bilinear_layers[i]), hd.head[i])
    raise NotImplementedError(f"head_type {hd.head_type!r}")


# ------------------------------------------------------------------------------------------------ window transformer
def window_block(blk, x, B, S):
    """VideoChapterBlock.forward (stacked_window_self_attention.py:128-145): x [B*S, H] -> [B*S, H]."""
    at = blk.attention
    n = layer_norm(x, blk.attention_norm)
    mid = S // 2
    # get_relative_positions :48-52, in fp32 as torch computes it
    pos = _positions((np.arange(S, dtype=np.float32) - np.float32(mid)) / np.float32(mid + 1e-6), x.device)
    n2 = PosEncFn.apply(n, at.position_encoding, pos)                          # hidden_states + position_emb
    q, k, v = linear(n2, at.query), linear(n2, at.key), linear(n2, at.value)
    ctx = MHAFn.apply(q, k, v, at.window_pos_bias, B, S, S, at.num_attention_heads, _drop_p(at.attention_dropout))
    x = linear(ctx, at.out_proj, res=x)                                            # attention_output + residual
    return chain(layer_norm(x, blk.ffn_norm), blk.ffn, res=x)                      # ffn_output + residual


def window_attention(wa, fusion_emb):
    """StackedVideoChapterAttention.forward (:204-223) in training: fusion_emb [B, S, H] -> logits [B, 2]."""
    B, S, H = fusion_emb.shape
    P_len = wa.layers[0].attention.window_pos_bias.shape[-1]
    if S > P_len:
        raise RuntimeError(f"window of {S} clips exceeds 2 * window_size + 1 = {P_len} (window_pos_bias length)")
    x = fusion_emb.reshape(B * S, H)
    for blk in wa.layers:
        x = window_block(blk, x, B, S)
    x = layer_norm(x, wa.final_layer_norm)
    target = x.view(B, S, H)[:, S // 2].contiguous()
    return chain(target, wa.classifier)
