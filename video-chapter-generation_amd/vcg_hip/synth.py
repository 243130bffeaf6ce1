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
