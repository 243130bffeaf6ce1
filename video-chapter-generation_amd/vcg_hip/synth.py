"""Seeded synthetic data: clip windows and weights.

`fill_np` is the numpy twin of the `vcg_synth` HIP kernel (csrc/synth.hip) and produces
bit-identical values; `fill_dev` runs the kernel so large tensors are generated directly in HBM.
Keys are derived from (seed, name) with FNV-1a so every tensor has an independent stream.
"""
import numpy as np

GOLDEN = np.uint64(0x9E3779B97F4A7C15)
M1 = np.uint64(0xBF58476D1CE4E5B9)
M2 = np.uint64(0x94D049BB133111EB)

KIND_UNIFORM, KIND_NORMAL, KIND_INT = 0, 1, 2


def key_of(seed, name):
    """FNV-1a 64 of f'{seed}:{name}'."""
    h = 0xCBF29CE484222325
    for b in f"{seed}:{name}".encode():
        h ^= b
        h = (h * 0x100000001B3) & 0xFFFFFFFFFFFFFFFF
    return h


def _mix64(z):
    z = (z ^ (z >> np.uint64(30))) * M1
    z = (z ^ (z >> np.uint64(27))) * M2
    return z ^ (z >> np.uint64(31))


def _hk(key, idx, k):
    return _mix64(np.uint64(key) + GOLDEN * (np.uint64(4) * idx + np.uint64(k + 1)))


def _u24(h):
    return (h >> np.uint64(40)).astype(np.float64) * (1.0 / 16777216.0)


def fill_np(n, kind, key, a, b, chunk=1 << 22):
    """Numpy reference of vcg_synth. Returns float32 (kinds 0/1) or int64 (kind 2)."""
    out = np.empty(n, dtype=np.int64 if kind == KIND_INT else np.float32)
    with np.errstate(over="ignore"):
        for s in range(0, n, chunk):
            idx = np.arange(s, min(n, s + chunk), dtype=np.uint64)
            if kind == KIND_INT:
                span = np.uint64(int(b) - int(a))
                h = _hk(key, idx, 0)
                out[s:s + len(idx)] = int(a) + ((h >> np.uint64(11)) % span).astype(np.int64)
            elif kind == KIND_UNIFORM:
                u = _u24(_hk(key, idx, 0))
                out[s:s + len(idx)] = (np.float64(a) + (np.float64(b) - np.float64(a)) * u).astype(np.float32)
            else:
                sm = _u24(_hk(key, idx, 0)) + _u24(_hk(key, idx, 1))
                sm = sm + _u24(_hk(key, idx, 2))
                sm = sm + _u24(_hk(key, idx, 3))
                z = (sm - 2.0) * 1.7320508075688772
                out[s:s + len(idx)] = (np.float64(a) + np.float64(b) * z).astype(np.float32)
    return out


def fill_dev(out, kind, key, a, b):
    """Fill a GPU tensor with the HIP generator (bit-identical to fill_np)."""
    from . import ops
    return ops.synth(out, kind, key, a, b)


def fill(t, kind, key, a, b):
    """Fill tensor `t` in place: HIP kernel on GPU tensors, numpy twin on CPU tensors."""
    import torch
    if t.is_cuda:
        if kind == KIND_INT:
            assert t.dtype == torch.int64
        else:
            assert t.dtype == torch.float32
        fill_dev(t, kind, key, a, b)
    else:
        v = fill_np(t.numel(), kind, key, a, b)
        t.copy_(torch.from_numpy(v).view(t.shape))
    return t


# ------------------------------------------------------------------------------ weights
def init_rule(name, shape):
    """(kind, a, b) for a TwoStream parameter name (reference state-dict naming).

    vision convs: N(0, sqrt(2/fan_out)) (torchvision kaiming fan_out); vision BN gamma U(0.5,1.5)
    (U(0.2,0.6) on bn3 / downsample.1 to keep the residual stream bounded), beta U(-0.2,0.2);
    BERT Linear/Embedding N(0, 0.02), biases N(0, 0.02), LayerNorm gamma U(0.8,1.2), beta U(-0.1,0.1);
    head Linear U(+-1/sqrt(fan_in)) (nn.Linear default bound)."""
    leaf = name.rsplit(".", 1)[-1]
    if name.startswith("window_attn."):  # StackedVideoChapterAttention (stacked_window_self_attention.py)
        if leaf == "window_pos_bias":
            return KIND_NORMAL, 0.0, 0.02
        if len(shape) == 2:  # Linear weight [out][in]: U(+-1/sqrt(fan_in)); Linear(1, H): U(+-1)
            bound = 1.0 / np.sqrt(shape[1])
            return KIND_UNIFORM, -bound, bound
        if leaf == "weight":  # every 1-D weight is a LayerNorm gamma
            return KIND_UNIFORM, 0.8, 1.2
        return KIND_UNIFORM, -0.1, 0.1  # Linear biases and LayerNorm betas
    if len(shape) == 4:
        fan_out = shape[0] * shape[2] * shape[3]
        return KIND_NORMAL, 0.0, float(np.sqrt(2.0 / fan_out))
    is_vision_bn = ("vision_model" in name or name.startswith(("bn", "layer"))) and len(shape) == 1 and (
        ".bn" in "." + name or "downsample.1" in name)
    if is_vision_bn:
        if leaf == "weight":
            small = ".bn3." in "." + name or "downsample.1" in name
            return (KIND_UNIFORM, 0.2, 0.6) if small else (KIND_UNIFORM, 0.5, 1.5)
        return KIND_UNIFORM, -0.2, 0.2
    if "LayerNorm" in name:
        return (KIND_UNIFORM, 0.8, 1.2) if leaf == "weight" else (KIND_UNIFORM, -0.1, 0.1)
    if "fusion_head" in name or name.startswith(("head.", "lang_proj_head", "vision_proj_head")):
        if len(shape) == 1 and leaf == "weight":  # LayerNorm gamma of the window ChapterHead's projection chains
            return KIND_UNIFORM, 0.8, 1.2
        fan_in = shape[-1] if len(shape) == 2 else None
        if fan_in is None:  # bias: bound from the matching weight's fan_in is not known here; use 1/sqrt(D)
            fan_in = max(1, shape[0])
        bound = 1.0 / np.sqrt(fan_in)
        return KIND_UNIFORM, -bound, bound
    return KIND_NORMAL, 0.0, 0.02


def init_params(module, seed=123, prefix=""):
    """Deterministically (re)initialise every parameter of `module` by name; works for CPU modules
    (numpy twin) and GPU modules (HIP generator) with bit-identical results."""
    import torch
    with torch.no_grad():
        for n, p in module.named_parameters():
            full = prefix + n
            kind, a, b = init_rule(full, tuple(p.shape))
            if p.is_cuda and p.is_contiguous():
                fill(p.data, kind, key_of(seed, full), a, b)
            else:
                v = fill_np(p.numel(), kind, key_of(seed, full), a, b)
                p.data.copy_(torch.from_numpy(v).view(p.shape))
            if full.endswith("word_embeddings.weight"):
                p.data[0].zero_()  # HF init zeroes the padding row (padding_idx = 0)
        for n, b in module.named_buffers():
            if n.endswith("running_mean"):
                b.zero_()
            elif n.endswith("running_var"):
                b.fill_(1.0)


def load_bn_stats(module, stats, prefix=""):
    """Copy running_mean / running_var from a {name: array} mapping (names relative to TwoStream)."""
    import torch
    with torch.no_grad():
        for n, b in module.named_buffers():
            full = prefix + n
            if full in stats and (n.endswith("running_mean") or n.endswith("running_var")):
                b.copy_(torch.as_tensor(np.asarray(stats[full])).to(b.device, b.dtype))


# ------------------------------------------------------------------------------ clip windows
def clip_batch(B, T, H, W, L, seed=123, device="cpu", vocab=30522):
    """Synthetic clip windows: frames ~ N(0,1) post-normalisation [B,T,3,H,W] f32,
    ids [B,L] (101 at 0, others uniform [1000, vocab)), n_valid uniform in [L/2, L], pad 0,
    mask 1/0, labels Bernoulli(0.5)."""
    import torch
    frames = torch.empty((B, T, 3, H, W), dtype=torch.float32, device=device)
    fill(frames, KIND_NORMAL, key_of(seed, "frames"), 0.0, 1.0)
    ids = torch.empty((B, L), dtype=torch.int64, device=device)
    fill(ids, KIND_INT, key_of(seed, "ids"), 1000, vocab)
    nval = fill_np(B, KIND_INT, key_of(seed, "n_valid"), L // 2, L + 1)
    lab = fill_np(B, KIND_INT, key_of(seed, "labels"), 0, 2)
    pos = np.arange(L)[None, :]
    mask_np = (pos < nval[:, None]).astype(np.int64)
    mask = torch.from_numpy(mask_np).to(device)
    ids[:, 0] = 101
    ids.mul_(mask)  # pad id 0 where mask == 0
    labels = torch.from_numpy(lab.astype(np.int64)).to(device)
    return frames, ids, mask, labels
