"""Single-model classification heads (reference Resnet50TSM.head resnet50_tsm.py:22-23,68-77 and
BertHugface.head bert_hugface.py:34-36,127-130): logits = x W^T + b, prob = softmax(logits, 1),
on the fused head kernel (T = 0 rows of vision features, i.e. a plain Linear)."""
import torch

from . import ops


class _LinearHeadFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias):
        x = x.contiguous()
        B, D = x.shape
        O = weight.shape[0]
        logits, prob = ops.head_mlp_fwd(x, x, weight, bias, B, 0, D, O)
        ctx.save_for_backward(x, weight, prob)
        ctx.has_bias = bias is not None
        ctx.bias = bias
        return logits, prob

    @staticmethod
    def backward(ctx, dlogits, dprob):
        x, weight, prob = ctx.saved_tensors
        if dlogits is None:
            dlogits = torch.zeros_like(prob)
        if dprob is not None:
            dlogits = dlogits + prob * (dprob - (dprob * prob).sum(1, keepdim=True))
        B, D = x.shape
        O = weight.shape[0]
        dW = torch.zeros_like(weight)
        db = torch.zeros(O, dtype=torch.float32, device=x.device)
        _, dx = ops.head_mlp_bwd(x, x, weight, dlogits.contiguous(), dW, db, B, 0, D, O, relu_mask=False)
        return dx, dW, (db if ctx.has_bias else None)


def linear_head(root, head, x):
    if head is None:
        raise RuntimeError("call build_chapter_head() first")
    if x.dtype != torch.float32:
        x = x.float()
    return _LinearHeadFn.apply(x, head.weight, head.bias)
