"""Fused AdamW over the flat parameter buffer (+ on-device gradient-norm clipping).

`configure_adamw` reproduces TwoStream.configure_optimizers' two parameter groups
(reference model/fusion/two_stream.py:127-169) and returns a `FusedAdamW`, a
torch.optim.Optimizer subclass with AdamW's param_groups / state_dict layout whose step is ONE
kernel over all parameters. `clip_and_step(max_norm)` fuses torch.nn.utils.clip_grad_norm_
(train_video_segment_point.py:204) into the same launch without a host synchronisation.
"""
import torch

from . import flat as flatmod
from . import ops


def _no_decay(full_name, leaf_name):
    """The reference grouping rule (two_stream.py:135-164, resnet50_tsm.py:35-65): biases, LayerNorm, BatchNorm
    ("bn") and embedding ("emb") parameters take no weight decay."""
    return leaf_name.endswith("bias") or any(tag in full_name for tag in ("LayerNorm", "bn", "emb"))


def param_groups(model, weight_decay):
    """[decay group, no-decay group] over every parameter, each sorted by name (the reference's order)."""
    named = dict(model.named_parameters())
    owner = {}  # full name -> decided by the module that owns it directly
    for mod_name, mod in model.named_modules():
        for leaf, _ in mod.named_parameters(recurse=False):
            full = f"{mod_name}.{leaf}" if mod_name else leaf
            owner[full] = _no_decay(full, leaf)
    unassigned = set(named) - set(owner)
    if unassigned:
        raise ValueError(f"param_groups: no owning module found for {sorted(unassigned)}")
    decay = sorted(n for n, nd in owner.items() if not nd and n in named)
    no_decay = sorted(n for n, nd in owner.items() if nd and n in named)
    return [
        {"params": [named[n] for n in decay], "weight_decay": weight_decay},
        {"params": [named[n] for n in no_decay], "weight_decay": 0.0},
    ]


def configure_adamw(model, train_config):
    groups = param_groups(model, train_config.weight_decay)
    return FusedAdamW(groups, lr=train_config.learning_rate, betas=train_config.betas, model=model)


class FusedAdamW(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2, model=None):
        defaults = dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay)
        super().__init__(params, defaults)
        self.model = model
        self._flat = None
        self._m = self._v = None
        self._flags = None
        self._step_count = 0
        self._sumsq = None
        self._sumsq_ws = None
        self.grad_scale = 1.0  # e.g. 1/world_size when gradients are all-reduced with SUM

    # ------------------------------------------------------------------ flat binding
    def _bind(self):
        model = self.model
        if model is None:
            raise RuntimeError("FusedAdamW needs the model (configure_optimizers passes it)")
        f = model.native_flat()
        if f is self._flat:
            return f
        params = [p for g in self.param_groups for p in g["params"]]
        if any(id(p) not in f.index for p in params):
            raise RuntimeError("optimizer parameters are not all in the model's flat buffer")
        g0 = self.param_groups[0]
        for g in self.param_groups:
            if (g["lr"], tuple(g["betas"]), g["eps"]) != (g0["lr"], tuple(g0["betas"]), g0["eps"]):
                raise NotImplementedError("FusedAdamW: all groups must share lr / betas / eps")
        wds = {g["weight_decay"] for g in self.param_groups if g["weight_decay"] != 0.0}
        if len(wds) > 1:
            raise NotImplementedError("FusedAdamW: at most one non-zero weight_decay value")
        self._wd = wds.pop() if wds else 0.0
        flags = torch.full((f.total // flatmod.ALIGN,), 2, dtype=torch.uint8)  # default: skipped
        for g in self.param_groups:
            code = 1 if g["weight_decay"] != 0.0 else 0
            for p in g["params"]:
                if not p.requires_grad:
                    continue
                o = f.offset_of(p)
                flags[o // flatmod.ALIGN:(o + p.numel() + flatmod.ALIGN - 1) // flatmod.ALIGN] = code
        self._flags = flags.to(f.device)
        old_m, old_v = self._m, self._v
        self._m = torch.zeros(f.total, dtype=torch.float32, device=f.device)
        self._v = torch.zeros(f.total, dtype=torch.float32, device=f.device)
        # carry over loaded / previous per-parameter state
        for p in params:
            st = self.state.get(p)
            if st and "exp_avg" in st:
                o = f.offset_of(p)
                self._m[o:o + p.numel()].copy_(st["exp_avg"].reshape(-1))
                self._v[o:o + p.numel()].copy_(st["exp_avg_sq"].reshape(-1))
        del old_m, old_v
        self._sumsq = torch.zeros(1, dtype=torch.float32, device=f.device)
        self._flat = f
        self._rebind_state()
        return f

    def _rebind_state(self):
        f = self._flat
        step_t = torch.tensor(float(self._step_count))
        for g in self.param_groups:
            for p in g["params"]:
                o = f.offset_of(p)
                self.state[p] = {"step": step_t,
                                 "exp_avg": self._m[o:o + p.numel()].view(p.shape),
                                 "exp_avg_sq": self._v[o:o + p.numel()].view(p.shape)}

    # ------------------------------------------------------------------ steps
    @torch.no_grad()
    def step(self, closure=None, max_norm=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        f = self._bind()
        self._step_count += 1
        g0 = self.param_groups[0]
        b1, b2 = g0["betas"]
        sumsq = None
        if max_norm is not None:
            self._sumsq_ws = ops.sumsq(f.grad, self._sumsq, self._sumsq_ws)
            sumsq = self._sumsq
        ops.adamw(f.data, f.grad, self._m, self._v, self._flags, flatmod.FLAG_SHIFT, g0["lr"], b1, b2, g0["eps"],
                  self._wd, self._step_count, sumsq, float(max_norm) if max_norm is not None else 1.0,
                  self.grad_scale, f.shadow)
        if f.shadow is not None:
            f.mark_shadow_current()
        step_t = torch.tensor(float(self._step_count))
        for p in self.state:
            self.state[p]["step"] = step_t
        return loss

    def clip_and_step(self, max_norm):
        """clip_grad_norm_(params, max_norm) + step, fused and host-sync free."""
        return self.step(max_norm=max_norm)

    def grad_norm(self):
        """Total gradient L2 norm (after grad_scale), as a device scalar."""
        f = self._bind()
        self._sumsq_ws = ops.sumsq(f.grad, self._sumsq, self._sumsq_ws)
        return self._sumsq.sqrt()[0] * self.grad_scale

    def zero_grad(self, set_to_none=True):
        if self.model is not None:
            self.model.zero_grad()
        else:
            super().zero_grad(set_to_none)

    def load_state_dict(self, state_dict):
        super().load_state_dict(state_dict)
        steps = [float(s["step"]) for s in self.state.values() if "step" in s]
        self._step_count = int(max(steps)) if steps else 0
        if self._flat is not None:
            f = self._flat
            for p, st in list(self.state.items()):
                if "exp_avg" in st:
                    o = f.offset_of(p)
                    self._m[o:o + p.numel()].copy_(st["exp_avg"].reshape(-1))
                    self._v[o:o + p.numel()].copy_(st["exp_avg_sq"].reshape(-1))
            self._rebind_state()
