"""autograd.Function glue: each Function runs a native engine forward and a hand-written native
backward. Parameters are not Function inputs; their gradients are accumulated by the kernels
directly into the flat .grad buffer. A zero-size `anchor` tensor (requires_grad) ties each
Function into the autograd graph so `loss.backward()` reaches it even when its inputs are integer
token ids or frames that need no gradient.
"""
import torch

from . import ops


class TrunkFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, anchor, engine, need_grad, hooks):
        ctx.set_materialize_grads(False)
        emb, saved = engine.forward(x, need_grad)
        ctx.engine, ctx.saved, ctx.hooks = engine, saved, hooks
        return emb

    @staticmethod
    def backward(ctx, d_emb):
        if ctx.saved is None:
            raise RuntimeError("TrunkFn: forward ran without saving activations (need_grad=False)")
        if d_emb is not None:
            ctx.engine.backward(d_emb, ctx.saved, hooks=ctx.hooks)
        ctx.saved = None
        return None, None, None, None, None


class BertFn(torch.autograd.Function):
    """BERT encoder. `join` (optional): the stream that consumes the outputs when the encoder runs on a side
    stream concurrently with the trunk (TwoStream.forward). Autograd runs the backward on the forward's stream
    (the side stream); it ends by making `join` wait for it, so the gradients are complete on the caller's
    stream when backward() returns."""

    @staticmethod
    def forward(ctx, ids, mask, anchor, engine, need_grad, seed, hooks, join=None):
        ctx.set_materialize_grads(False)
        pooled, last, saved = engine.forward(ids, mask, need_grad, seed)
        ctx.engine, ctx.saved, ctx.hooks, ctx.join = engine, saved, hooks, join
        if pooled is None:
            pooled = torch.zeros(0, device=ids.device)
        return pooled, last

    @staticmethod
    def backward(ctx, d_pooled, d_last):
        if ctx.saved is None:
            raise RuntimeError("BertFn: forward ran without saving activations (need_grad=False)")
        if ctx.join is not None:  # incoming grads were made on the joining stream: keep their memory alive here
            cur = torch.cuda.current_stream()
            for t in (d_pooled, d_last):
                if t is not None and t.is_cuda:
                    t.record_stream(cur)
        if d_pooled is not None or d_last is not None:
            ctx.engine.backward(d_pooled if d_pooled is not None and d_pooled.numel() else None, d_last, ctx.saved,
                                hooks=ctx.hooks)
        ctx.saved = None
        if ctx.join is not None:
            ctx.join.wait_stream(torch.cuda.current_stream())
        return None, None, None, None, None, None, None, None


class HeadFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, lang, vis, anchor, engine, need_grad, hooks):
        ctx.set_materialize_grads(False)
        logits, prob, saved = engine.forward(lang, vis, need_grad)
        ctx.engine, ctx.saved, ctx.hooks = engine, saved, hooks
        ctx.save_for_backward(prob)
        return logits, prob

    @staticmethod
    def backward(ctx, dlogits, dprob):
        if ctx.saved is None:
            raise RuntimeError("HeadFn: forward ran without saving activations (need_grad=False)")
        (prob,) = ctx.saved_tensors
        if dlogits is None:
            dlogits = torch.zeros_like(prob)
        if dprob is not None:
            # softmax backward for a gradient through the returned probabilities (2-wide, host-light)
            dlogits = dlogits + prob * (dprob - (dprob * prob).sum(1, keepdim=True))
        dlang, dvis = ctx.engine.backward(dlogits, ctx.saved)
        ctx.saved = None
        if ctx.hooks is not None:
            ctx.hooks(list(ctx.engine.h.parameters()))
        return dlang, dvis, None, None, None, None


def cross_entropy(logits, labels):
    """Mean cross-entropy (F.cross_entropy, train_video_segment_point.py:165): the vcg::cross_entropy torch.library
    op (vcg_hip/torch_ops.py) over vcg_cross_entropy_fwd / _bwd."""
    from . import torch_ops  # noqa: F401  (registers torch.ops.vcg.*)
    return torch.ops.vcg.cross_entropy(logits, labels.to(torch.int64))
