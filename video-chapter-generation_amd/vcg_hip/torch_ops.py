"""libvcg_hip entry points registered as torch.library custom ops (namespace `vcg`), the op surface SURVEY §8b
names for the model/ and ops/ wrappers: each op has a schema, a fake (meta) implementation for shape inference /
tracing, and, where the reference op is differentiable, an autograd formula that is itself a vcg op.

    vcg::tsm_shift(x, n_segment, fold_div, direction)      TemporalShift.shift (ops/temporal_shift.py:33-51) and
                                                           its adjoint (direction 1); ops/temporal_shift.py calls it
    vcg::cross_entropy(logits, labels) / _bwd              F.cross_entropy (train_video_segment_point.py:165);
                                                           vcg_hip.functions.cross_entropy calls it
    vcg::window_frames_u8(frames, idx, bf16, cpad)         the frame ingest (gather + ToTensor + Normalize into the
                                                           stem layout, youtube_dataset.py:180-190)
    vcg::linear(x, weight, bias, act)                      nn.Linear (+ ReLU / GELU / tanh epilogue) on the GEMM engine;
                                                           differentiable without an activation (any dtype) and with
                                                           ReLU (fp32): dX = dY' W, dW = dY'^T X, db = colsum(dY');
                                                           GELU / tanh epilogues are forward-only (backward raises)

The encoder engines (vcg_hip/trunk.py, bert.py) issue ~2000 launches per train step and call the C ABI through
ctypes directly: a dispatcher round trip per launch (~5-10 us of host time) would make the step host-bound.
"""
from typing import Optional, Tuple

import torch

from . import ops

_DT = {False: torch.float32, True: torch.bfloat16}


@torch.library.custom_op("vcg::tsm_shift", mutates_args=())
def tsm_shift(x: torch.Tensor, n_segment: int, fold_div: int, direction: int) -> torch.Tensor:
    if x.dim() != 4 or x.shape[0] % n_segment != 0:
        raise RuntimeError(f"vcg::tsm_shift: x must be [n_batch*{n_segment}, C, H, W], got {tuple(x.shape)}")
    return ops.tsm_shift(x.contiguous(), n_segment, fold_div, direction=direction)


@tsm_shift.register_fake
def _(x, n_segment, fold_div, direction):
    return x.new_empty(x.shape)  # (contiguous, as the real op returns)


def _tsm_setup(ctx, inputs, output):
    _, ctx.n_segment, ctx.fold_div, ctx.direction = inputs


def _tsm_backward(ctx, g):
    return torch.ops.vcg.tsm_shift(g, ctx.n_segment, ctx.fold_div, 1 - ctx.direction), None, None, None


tsm_shift.register_autograd(_tsm_backward, setup_context=_tsm_setup)


@torch.library.custom_op("vcg::cross_entropy_bwd", mutates_args=())
def cross_entropy_bwd(logits: torch.Tensor, labels: torch.Tensor, dloss: torch.Tensor) -> torch.Tensor:
    return ops.cross_entropy_bwd(logits.contiguous(), labels.to(torch.int64).contiguous(), dloss.contiguous())


@cross_entropy_bwd.register_fake
def _(logits, labels, dloss):
    return torch.empty_like(logits)


@torch.library.custom_op("vcg::cross_entropy", mutates_args=())
def cross_entropy(logits: torch.Tensor, labels: torch.Tensor) -> torch.Tensor:
    if logits.dim() != 2 or labels.shape != logits.shape[:1]:
        raise RuntimeError("vcg::cross_entropy: logits [B, C] and labels [B]")
    return ops.cross_entropy_fwd(logits.contiguous(), labels.to(torch.int64).contiguous())


@cross_entropy.register_fake
def _(logits, labels):
    return logits.new_empty(())


def _ce_setup(ctx, inputs, output):
    ctx.save_for_backward(*inputs)


def _ce_backward(ctx, dloss):
    logits, labels = ctx.saved_tensors
    return torch.ops.vcg.cross_entropy_bwd(logits, labels, dloss), None


cross_entropy.register_autograd(_ce_backward, setup_context=_ce_setup)


@torch.library.custom_op("vcg::window_frames_u8", mutates_args=())
def window_frames_u8(frames: torch.Tensor, idx: torch.Tensor, bf16: bool, cpad: int) -> torch.Tensor:
    return ops.window_frames_u8(frames, idx.contiguous(), _DT[bf16], cpad=cpad)


@window_frames_u8.register_fake
def _(frames, idx, bf16, cpad):
    F, H, W, _ = frames.shape
    return frames.new_empty((idx.numel(), H, W, cpad), dtype=_DT[bf16])


@torch.library.custom_op("vcg::linear", mutates_args=())
def linear(x: torch.Tensor, weight: torch.Tensor, bias: Optional[torch.Tensor], act: int) -> torch.Tensor:
    if x.dim() != 2 or weight.dim() != 2 or x.shape[1] != weight.shape[1] or x.dtype != weight.dtype:
        raise RuntimeError("vcg::linear: x [M, K] and weight [N, K] of one dtype")
    M, K = x.shape
    N = weight.shape[0]
    return ops.gemm(x.contiguous(), weight.contiguous(), M, N, K, K, K, bias=bias, act=act)


@linear.register_fake
def _(x, weight, bias, act):
    return x.new_empty((x.shape[0], weight.shape[0]))


@torch.library.custom_op("vcg::linear_bwd", mutates_args=())
def linear_bwd(dy: torch.Tensor, x: torch.Tensor, weight: torch.Tensor, out: Optional[torch.Tensor], act: int,
               has_bias: bool) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    """(dx, dW, db) of vcg::linear; db is [N] fp32 (empty without a bias). ReLU: the mask from the saved output."""
    M, K = x.shape
    N = weight.shape[0]
    dy = dy.contiguous()
    if act == ops.ACT_RELU:
        if dy.dtype != torch.float32:
            raise NotImplementedError("vcg::linear backward through ReLU: fp32 only (vcg_act_drop_bwd)")
        dpre = torch.empty_like(dy)
        ops._lib.call("vcg_act_drop_bwd", ops.P(dy), ops.P(out.contiguous()), ops.P(dpre), dy.numel(), ops.ACT_RELU,
                      0.0, 0, ops.stream())
        dy = dpre
    elif act != ops.ACT_NONE:
        raise NotImplementedError(f"vcg::linear backward: act {act} is forward-only (no pre-activation saved)")
    dx = ops.gemm(dy, weight.contiguous(), M, K, N, N, K, transB=True)
    # dW = dY^T X over the M rows: the split-K engine (fp32 slabs, any M), rounded to the weight's dtype
    dw32 = torch.empty((N, K), dtype=torch.float32, device=dy.device)
    ops.gemm_splitk(dy, x.contiguous(), dw32, N, K, M, N, K, transA=True, transB=True, accumulate=False)
    dw = dw32.to(weight.dtype)
    db = torch.empty(N if has_bias else 0, dtype=torch.float32, device=dy.device)
    if has_bias:
        ops.colsum(dy, N, M, N, db, accumulate=False)
    return dx, dw, db


@linear_bwd.register_fake
def _(dy, x, weight, out, act, has_bias):
    N = weight.shape[0]
    return (x.new_empty(x.shape), weight.new_empty(weight.shape),
            dy.new_empty((N if has_bias else 0,), dtype=torch.float32))


def _linear_setup(ctx, inputs, output):
    x, weight, bias, act = inputs
    ctx.act, ctx.has_bias = act, bias is not None
    ctx.bias_dtype = bias.dtype if bias is not None else None
    ctx.save_for_backward(x, weight, output if act == ops.ACT_RELU else None)


def _linear_backward(ctx, dy):
    x, weight, out = ctx.saved_tensors
    dx, dw, db = torch.ops.vcg.linear_bwd(dy, x, weight, out, ctx.act, ctx.has_bias)
    return dx, dw, (db.to(ctx.bias_dtype) if ctx.has_bias else None), None


linear.register_autograd(_linear_backward, setup_context=_linear_setup)
