"""Flat parameter / gradient storage.

All fp32 master parameters of a model live in ONE contiguous HBM buffer (each tensor 256-element
aligned), their `.grad` tensors are views into ONE flat gradient buffer, and (bf16 mode) a bf16
shadow copy of the parameters is kept in a third flat buffer that the fused AdamW kernel refreshes
as it updates. This is what lets one kernel clip + update all 133 M parameters, lets the gradient
all-reduce run over large contiguous buckets, and gives BERT's fused QKV weight as a plain view.

Parameter objects keep their identity (`p.data` is re-pointed), so state dicts, optimizers and
`named_parameters()` behave exactly like the reference modules'.
"""
import torch

from . import ops

ALIGN = 256  # elements (1 KiB); also the granularity of the weight-decay flag table
FLAG_SHIFT = 8


def no_decay_name(name):
    """TwoStream.configure_optimizers grouping (reference model/fusion/two_stream.py:135-152)."""
    pn = name.rsplit(".", 1)[-1]
    if pn.endswith("bias"):
        return True
    if "LayerNorm" in name or "bn" in name or "emb" in name:
        return True
    return False


class FlatParams:
    def __init__(self, named_params, device, shadow_dtype=None, order=None):
        """named_params: list of (name, Parameter). `order` (optional) is a list of names giving the
        layout order; params not listed keep their relative order after the listed ones."""
        self.device = torch.device(device)
        named = list(named_params)
        if order is not None:
            pos = {n: i for i, n in enumerate(order)}
            named.sort(key=lambda kv: (pos.get(kv[0], len(pos)), ))
        self.names = [n for n, _ in named]
        self.params = [p for _, p in named]
        self.offsets = []
        off = 0
        for p in self.params:
            self.offsets.append(off)
            off += (p.numel() + ALIGN - 1) // ALIGN * ALIGN
        self.total = off
        self.data = torch.zeros(self.total, dtype=torch.float32, device=self.device)
        self.grad = torch.zeros(self.total, dtype=torch.float32, device=self.device)
        flags = torch.zeros(self.total // ALIGN, dtype=torch.uint8)
        for n, p, o in zip(self.names, self.params, self.offsets):
            self.data[o:o + p.numel()].copy_(p.detach().reshape(-1).to(self.device))
            if not no_decay_name(n):
                flags[o // ALIGN:(o + p.numel() + ALIGN - 1) // ALIGN] = 1
        self.wd_flags = flags.to(self.device)
        for p, o in zip(self.params, self.offsets):
            p.data = self.data[o:o + p.numel()].view(p.shape)
            p.grad = self.grad[o:o + p.numel()].view(p.shape)
        self.index = {id(p): i for i, p in enumerate(self.params)}
        self.shadow_dtype = shadow_dtype
        self.shadow = None
        self._shadow_version = None
        if shadow_dtype is not None and shadow_dtype != torch.float32:
            self.shadow = torch.empty(self.total, dtype=shadow_dtype, device=self.device)

    # ------------------------------------------------------------------ validity
    def intact(self):
        """True if every parameter is still a view of the flat buffers (no .to()/reassignment)."""
        base = self.data.data_ptr()
        gbase = self.grad.data_ptr()
        for p, o in zip(self.params, self.offsets):
            if p.data.data_ptr() != base + 4 * o:
                return False
            if p.grad is None or p.grad.data_ptr() != gbase + 4 * o:
                return False
        return True

    def rebind_grads(self):
        for p, o in zip(self.params, self.offsets):
            p.grad = self.grad[o:o + p.numel()].view(p.shape)

    def zero_grad(self):
        self.rebind_grads()
        self.grad.zero_()

    # ------------------------------------------------------------------ views
    def offset_of(self, p):
        return self.offsets[self.index[id(p)]]

    def contiguous_view(self, plist, shape, which="data"):
        """View over several parameters laid out back to back (e.g. fused QKV)."""
        o0 = self.offset_of(plist[0])
        n = 0
        for p in plist:
            assert self.offset_of(p) == o0 + n, "parameters are not contiguous in the flat buffer"
            n += p.numel()
        buf = {"data": self.data, "grad": self.grad, "shadow": self.shadow}[which]
        return buf[o0:o0 + n].view(shape)

    def grad_of(self, p):
        o = self.offset_of(p)
        return self.grad[o:o + p.numel()].view(p.shape)

    def compute_view(self, p, dtype):
        """Parameter in the compute storage dtype (fp32 master or bf16 shadow). The caller refreshes
        the shadow once per forward (refresh_shadow)."""
        if dtype == torch.float32:
            return p.data
        o = self.offset_of(p)
        return self.shadow[o:o + p.numel()].view(p.shape)

    def compute_contiguous(self, plist, shape, dtype):
        if dtype == torch.float32:
            return self.contiguous_view(plist, shape, "data")
        return self.contiguous_view(plist, shape, "shadow")

    # ------------------------------------------------------------------ bf16 shadow
    def _version(self):
        return sum(p._version for p in self.params)

    # `generation` changes whenever the master weights may have changed (a fused optimizer step, an in-place
    # write seen through the tensors' version counters): derived weight layouts (the trunk's bf16 conv GEMM
    # operands) are rebuilt when it moves.
    generation = 0

    def refresh_shadow(self, force=False):
        if self.shadow is None:
            return
        v = self._version()
        if force or v != self._shadow_version:
            ops.cast_from_f32(self.data, self.shadow.dtype, out=self.shadow)
            self._shadow_version = v
            self.generation += 1

    def mark_shadow_current(self):
        """Called by the fused optimizer, which rewrote the shadow while updating."""
        self._shadow_version = self._version()
        self.generation += 1
