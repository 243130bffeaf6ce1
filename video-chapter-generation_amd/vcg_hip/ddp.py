"""Data-parallel gradient exchange: RCCL all-reduce over xGMI, overlapped with the backward.

Replaces the NCCL DDP of reference train_video_segment_ddp.py:131-148 (DDP(model) with 25 MB
buckets firing on every backward). One process per GPU; the flat fp32 gradient buffer is reduced
in contiguous buckets as soon as the native backward reports a group of parameters final (per
BERT layer, per ResNet block, head, embeddings). torch.distributed's "nccl" backend is RCCL on
ROCm; each collective runs on RCCL's own stream after an event wait on the compute stream, so the
exchange of layer i overlaps the backward of layer i-1. Reductions are SUM; the 1/world average
is folded into the fused optimizer (FusedAdamW.grad_scale) so no extra pass over the grads runs.
Skipping reductions on accumulation micro-steps (no_sync semantics) is `reducer.enabled = False`.
"""
import os

import torch
import torch.distributed as dist


_DEBUG = os.environ.get("VCG_DDP_DEBUG", "")


def _sid(stream):
    return None if stream is None else stream.cuda_stream


class GradAllReducer:
    def __init__(self, flat, bucket_bytes=64 << 20, group=None):
        self.flat = flat
        self.bucket_elems = max(1, bucket_bytes // 4)
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.enabled = self.world > 1
        self._lo = self._hi = None
        self._works = []
        self._done_lo = None
        self._stream = None  # stream the open bucket's gradients were produced on

    # called by the engines (autograd backward thread) with parameters whose grads are final
    def __call__(self, params):
        if not self.enabled or not params:
            return
        if isinstance(params, str):
            return
        f = self.flat
        lo = min(f.offset_of(p) for p in params)
        hi = max(f.offset_of(p) + p.numel() for p in params)
        hi = (hi + 255) // 256 * 256
        stream = torch.cuda.current_stream() if torch.cuda.is_available() and f.grad.is_cuda else None
        if _DEBUG:
            print(f"[ddp] hook stream={stream.cuda_stream if stream is not None else None} [{lo},{hi}) "
                  f"open={self._lo},{self._hi} on {self._stream.cuda_stream if self._stream is not None else None}",
                  flush=True)
        # the encoders' backwards run on two streams: a bucket never spans both (compare the raw handles:
        # torch.cuda.Stream's != against None is not reliable)
        if _sid(stream) != _sid(self._stream):
            self._flush()
            self._stream = stream
        if self._lo is not None and (hi == self._lo or lo == self._hi):
            self._lo, self._hi = min(lo, self._lo), max(hi, self._hi)
        else:
            self._flush()
            self._lo, self._hi = lo, hi
        if self._hi - self._lo >= self.bucket_elems:
            self._flush()

    def _flush(self):
        if self._lo is None:
            return
        buf = self.flat.grad[self._lo:min(self._hi, self.flat.total)]
        if _DEBUG:
            print(f"[ddp] flush [{self._lo},{self._hi}) bucket stream "
                  f"{self._stream.cuda_stream if self._stream is not None else None} current "
                  f"{torch.cuda.current_stream().cuda_stream}", flush=True)
            if _DEBUG == "sync":
                (self._stream or torch.cuda.current_stream()).synchronize()
        if self._stream is not None and _sid(self._stream) != _sid(torch.cuda.current_stream()):
            with torch.cuda.stream(self._stream):  # the collective waits on the stream that made the bucket
                self._works.append(dist.all_reduce(buf, op=dist.ReduceOp.SUM, group=self.group, async_op=True))
        else:
            self._works.append(dist.all_reduce(buf, op=dist.ReduceOp.SUM, group=self.group, async_op=True))
        self._lo = self._hi = None

    def finish(self):
        """Flush the last bucket and make the current stream wait for every collective."""
        if not self.enabled:
            return
        self._flush()
        for w in self._works:
            w.wait()
        self._works = []

    def reduce_all(self):
        """Synchronous fallback: one all-reduce of the whole flat gradient buffer."""
        if self.enabled:
            dist.all_reduce(self.flat.grad, op=dist.ReduceOp.SUM, group=self.group)


def broadcast_parameters(model, src=0, group=None):
    """Rank-0 parameters / buffers to every rank (reference train_video_segment_ddp.py:261-263),
    one collective over the flat parameter buffer."""
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return
    f = model.native_flat()
    dist.broadcast(f.data, src=src, group=group)
    for b in model.buffers():
        if b is not None and b.is_floating_point():
            dist.broadcast(b, src=src, group=group)
    f.refresh_shadow(force=True)


def all_gather_object(obj, group=None):
    """Scalar gather for validation metrics (train_video_segment_ddp.py:278)."""
    if not dist.is_initialized():
        return [obj]
    out = [None] * dist.get_world_size(group)
    dist.all_gather_object(out, obj, group=group)
    return out
