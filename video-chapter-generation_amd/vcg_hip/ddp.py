"""Data-parallel gradient exchange: RCCL all-reduce over xGMI, overlapped with the backward.

Replaces the NCCL DDP of reference train_video_segment_ddp.py:131-148 (DDP(model) with 25 MB
buckets firing on every backward). One process per GPU; the flat fp32 gradient buffer is reduced
in contiguous buckets (25 MB by default, as DDP) as soon as the native backward reports a group of
parameters final (per BERT layer, per ResNet block, head, embeddings). Two transports:
  * torch.distributed (default): the "nccl" backend is RCCL on ROCm; each collective runs on RCCL's
    own stream after an event wait on the producing stream;
  * `comm=NativeComm(...)` (vcg_hip/comm.py): libvcg_hip's own RCCL C ABI (vcg_allreduce_bucket),
    issued on a side HIP stream that waits for the bucket's producer; finish() joins it.
Either way the exchange of layer i overlaps the backward of layer i-1. Reductions are SUM; the 1/world
average is folded into the fused optimizer (FusedAdamW.grad_scale) so no extra pass over the grads runs.
`wire_dtype=torch.bfloat16` halves the bytes on xGMI (267 MB instead of 533 MB per step): each bucket
is cast to bf16 on its producing stream, reduced, and cast back into the fp32 gradient at finish().
Skipping reductions on accumulation micro-steps (no_sync semantics) is `reducer.enabled = False`.
`record=True` keeps a log of hook calls and bucket flushes (the overlap evidence of tests/test_*_ddp.py).
"""
import os

import torch
import torch.distributed as dist


_DEBUG = os.environ.get("VCG_DDP_DEBUG", "")


class _nullctx:
    def __enter__(self):
        return None

    def __exit__(self, *a):
        return False


def _sid(stream):
    return None if stream is None else stream.cuda_stream


class GradAllReducer:
    def __init__(self, flat, bucket_bytes=25 << 20, group=None, wire_dtype=None, comm=None, record=False):
        self.flat = flat
        self.bucket_elems = max(1, bucket_bytes // 4)
        self.group = group
        self.world = comm.world if comm is not None else (dist.get_world_size(group) if dist.is_initialized() else 1)
        self.enabled = self.world > 1
        self.comm = comm
        if wire_dtype not in (None, torch.float32, torch.bfloat16):
            raise ValueError("wire_dtype must be None / torch.float32 / torch.bfloat16")
        self.wire = None if wire_dtype in (None, torch.float32) else wire_dtype
        self._wire_buf = None
        self._pending_casts = []  # (fp32 view, wire view) to cast back at finish()
        self._lo = self._hi = None
        self._works = []
        self._stream = None  # stream the open bucket's gradients were produced on
        self._side = None    # NativeComm: the side stream the collectives run on
        self.record = record
        self.log = []        # ("hook", lo, hi) / ("flush", lo, hi) in call order (record=True)
        self._flushed = []   # [lo, hi) ranges reduced in this backward: finish() reduces the rest of the buffer
        self._buckets = self._bytes = 0
        self.last_step = {"buckets": 0, "bytes": 0}  # collectives issued by the last finish()ed backward

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
        if self.record:
            self.log.append(("hook", lo, hi))
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

    def _wire_view(self, lo, hi):
        if self._wire_buf is None:
            self._wire_buf = torch.empty(self.flat.total, dtype=self.wire, device=self.flat.grad.device)
        return self._wire_buf[lo:hi]

    def _flush(self):
        if self._lo is None:
            return
        lo, hi = self._lo, min(self._hi, self.flat.total)
        self._flushed.append((lo, hi))
        buf = self.flat.grad[lo:hi]
        self._buckets += 1
        self._bytes += (hi - lo) * (2 if self.wire is not None else 4)
        if self.record:
            self.log.append(("flush", lo, hi))
        if _DEBUG:
            print(f"[ddp] flush [{lo},{hi}) bucket stream "
                  f"{self._stream.cuda_stream if self._stream is not None else None} current "
                  f"{torch.cuda.current_stream().cuda_stream}", flush=True)
            if _DEBUG == "sync":
                (self._stream or torch.cuda.current_stream()).synchronize()
        prod = self._stream
        cur = torch.cuda.current_stream() if buf.is_cuda else None
        with torch.cuda.stream(prod) if (prod is not None and _sid(prod) != _sid(cur)) else _nullctx():
            if self.wire is not None:  # cast on the producing stream (ordered after the bucket's kernels)
                wbuf = self._wire_view(lo, hi)
                if buf.is_cuda:
                    from . import ops
                    ops.cast_from_f32(buf, self.wire, out=wbuf)
                else:
                    wbuf.copy_(buf)
                self._pending_casts.append((buf, wbuf))
                buf = wbuf
            if self.comm is not None:
                if self._side is None:
                    self._side = torch.cuda.Stream(device=buf.device)
                self._side.wait_stream(torch.cuda.current_stream())  # the side stream waits for the producer
                self.comm.all_reduce(buf, stream=self._side)
            else:
                self._works.append(dist.all_reduce(buf, op=dist.ReduceOp.SUM, group=self.group, async_op=True))
        self._lo = self._hi = None

    def _gaps(self):
        """[lo, hi) ranges of the flat buffer no hook reported in this backward (parameters whose gradients are
        produced outside the native engines' reports, e.g. the window model's heads), coalesced."""
        out, pos = [], 0
        for lo, hi in sorted(self._flushed):
            if lo > pos:
                out.append((pos, lo))
            pos = max(pos, hi)
        if pos < self.flat.total:
            out.append((pos, self.flat.total))
        return out

    def finish(self):
        """Flush the last bucket, reduce every range no hook reported (so the whole gradient is always averaged,
        as DDP does), and make the current stream wait for every collective."""
        if not self.enabled:
            return
        self._flush()
        self._stream = torch.cuda.current_stream() if self.flat.grad.is_cuda else None
        for lo, hi in self._gaps():
            for b in range(lo, hi, self.bucket_elems):
                self._lo, self._hi = b, min(hi, b + self.bucket_elems)
                self._flush()
        self._flushed = []
        for w in self._works:
            w.wait()
        self._works = []
        if self._side is not None:
            torch.cuda.current_stream().wait_stream(self._side)
        for dst, src in self._pending_casts:  # bf16 wire -> the fp32 gradient (current stream, after the waits)
            if dst.is_cuda:
                from . import ops
                ops.cast_to_f32(src, out=dst)
            else:
                dst.copy_(src)
        self._pending_casts = []
        self.last_step = {"buckets": self._buckets, "bytes": self._bytes}
        self._buckets = self._bytes = 0

    def reduce_all(self):
        """Synchronous fallback: one all-reduce of the whole flat gradient buffer."""
        if self.enabled:
            dist.all_reduce(self.flat.grad, op=dist.ReduceOp.SUM, group=self.group)


def params_max_divergence(flat, src=0, group=None):
    """max over ranks and elements of |param - rank src's param| over the flat parameter buffer (0.0: every rank
    holds bit-identical parameters, as DDP guarantees after each synchronised step)."""
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return 0.0
    ref = flat.data.clone()
    dist.broadcast(ref, src=src, group=group)
    d = (flat.data - ref).abs().max().reshape(1).to(torch.float64)
    dist.all_reduce(d, op=dist.ReduceOp.MAX, group=group)
    return float(d.item())


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


class BufferBroadcaster:
    """DDP's broadcast_buffers=True (the default of the reference's DDP(model), train_video_segment_ddp.py:148):
    before every training forward, rank 0's floating-point buffers (BatchNorm running_mean / running_var) are
    copied to every rank, so the running statistics do not drift apart across ranks (each rank's BN sees only its
    own shard). The module buffers are re-bound to views of one flat buffer per dtype, so a sync is one collective
    per dtype. A buffer that was replaced since (model.to(), reassignment) is re-bound before the sync."""

    def __init__(self, model, src=0, group=None, comm=None):
        self.src, self.group, self.comm = src, group, comm
        self.model = model
        self.flats = {}
        self._bind()

    def _bufs(self):
        return [(m, n, b) for m in self.model.modules() for n, b in m._buffers.items()
                if b is not None and b.is_floating_point()]

    def _bind(self):
        bufs = self._bufs()
        self.flats, self.bound = {}, []
        for dt in dict.fromkeys(b.dtype for _, _, b in bufs):
            group = [(m, n, b) for m, n, b in bufs if b.dtype == dt]
            flat = torch.empty(sum(b.numel() for _, _, b in group), dtype=dt, device=group[0][2].device)
            o = 0
            for m, n, b in group:
                v = flat[o:o + b.numel()].view_as(b)
                v.copy_(b)
                m._buffers[n] = v
                self.bound.append((m, n, v))
                o += b.numel()
            self.flats[dt] = flat

    @property
    def flat(self):
        """The flat buffer of the (single) buffer dtype, None without floating buffers."""
        return next(iter(self.flats.values())) if len(self.flats) == 1 else (None if not self.flats else self.flats)

    def _intact(self):
        return all(m._buffers.get(n) is v for m, n, v in self.bound) and len(self.bound) == len(self._bufs())

    def __call__(self):
        if not self._intact():
            self._bind()
        for flat in self.flats.values():
            if self.comm is not None:
                self.comm.broadcast(flat, root=self.src)
            elif dist.is_initialized() and dist.get_world_size(self.group) > 1:
                dist.broadcast(flat, src=self.src, group=self.group)


def all_gather_object(obj, group=None):
    """Scalar gather for validation metrics (train_video_segment_ddp.py:278)."""
    if not dist.is_initialized():
        return [obj]
    out = [None] * dist.get_world_size(group)
    dist.all_gather_object(out, obj, group=group)
    return out
