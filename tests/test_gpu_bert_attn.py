"""Fused BERT self-attention (bert_attn.hip, the bf16 path) against an fp64 torch statement of HF BertSelfAttention
(eager: scores * scale + (1 - mask) * finfo(f32).min, softmax, dropout, PV; bert_hugface.py:20 -> BertModel) and
against the unfused kernels (QK^T GEMM -> attn_softmax -> PV GEMM) it replaces. The dropout mask is the library's
counter hash, restated in numpy here, so the fp64 reference drops exactly the same probabilities.

Tolerance (bf16 operands, fp32 accumulation): relative Frobenius error of ctx / dQ / dK / dV vs fp64 <= 2e-2, and
no worse than 1.25 x the unfused bf16 path's own error + 2e-3."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda"


def keep_mask(seed, idx, p):
    """common.h dropout_keep, vectorised (uint32 wrap-around arithmetic)."""
    if p <= 0:
        return np.ones(idx.shape, bool)
    with np.errstate(over="ignore"):
        h = (idx.astype(np.uint64) & np.uint64(0xFFFFFFFF)).astype(np.uint32) * np.uint32(0x9E3779B1)
        h ^= np.uint32(seed & 0xFFFFFFFF)
        h += np.uint32((seed >> 32) & 0xFFFFFFFF)
        h ^= h >> np.uint32(16)
        h *= np.uint32(0x85EBCA6B)
        h ^= h >> np.uint32(13)
        h *= np.uint32(0xC2B2AE35)
        h ^= h >> np.uint32(16)
    return (h >> np.uint32(8)).astype(np.float32) * np.float32(1.0 / 16777216.0) >= np.float32(p)


def ref_attention(qkv, mask, dctx, B, nh, L, Lp, p, seed):
    H = nh * 64
    x = qkv[:B * L].double().cpu().view(B, L, 3, nh, 64).permute(2, 0, 3, 1, 4)  # [3, B, nh, L, 64]
    q, k, v = (t.clone().requires_grad_(True) for t in x)
    add = (1.0 - mask.double().cpu())[:, None, None, :] * torch.finfo(torch.float32).min
    P = torch.softmax(q @ k.transpose(-1, -2) / 8.0 + add, dim=-1)
    z = np.arange(B * nh)[:, None, None]
    qi = np.arange(L)[None, :, None]
    kj = np.arange(L)[None, None, :]
    keep = torch.from_numpy(keep_mask(seed, (z * L + qi) * Lp + kj, p)).view(B, nh, L, L)
    Pd = P * keep / (1.0 - p)
    o = Pd @ v
    do = dctx.double().cpu().view(B, L, nh, 64).permute(0, 2, 1, 3)
    (o * do).sum().backward()
    ctx = o.permute(0, 2, 1, 3).reshape(B * L, H)
    dqkv = torch.stack([q.grad, k.grad, v.grad]).permute(1, 3, 0, 2, 4).reshape(B * L, 3 * H)
    return ctx, dqkv


def rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).norm() / b.norm()).item()


@pytest.mark.parametrize("B,L,p", [(3, 128, 0.0), (3, 128, 0.1), (2, 32, 0.1), (2, 100, 0.1), (1, 7, 0.0)])
def test_fused_attention_matches_fp64_and_unfused(B, L, p):
    from vcg_hip import _lib
    from vcg_hip.bert import attention_bwd, attention_fwd
    _lib.call("vcg_init", 0)
    nh, H = 12, 768
    Lp = (L + 7) // 8 * 8
    g = torch.Generator().manual_seed(B * 1000 + L)
    qkv = (torch.randn(B * L + 8, 3 * H, generator=g) * 1.5).to(torch.bfloat16).to(DEV)
    mask = torch.ones(B, L, dtype=torch.int64)
    mask[0, L - L // 3:] = 0          # padded keys
    if B > 1:
        mask[1, :] = 0                # a zero-padding clip: every key masked -> uniform rows (HF finfo.min)
    mask = mask.to(DEV)
    dctx = torch.randn(B * L, H, generator=g).to(torch.bfloat16).to(DEV)
    seed = 0x1234567890AB + L
    ref_ctx, ref_dqkv = ref_attention(qkv, mask, dctx, B, nh, L, Lp, p, seed)
    out = {}
    for fused in (True, False):
        ctx, att = attention_fwd(qkv, mask, B, nh, L, Lp, 64, 0.125, p, seed, fused)
        dqkv = attention_bwd(qkv, dctx, ctx, mask, att, B, nh, L, Lp, 64, 0.125, p, seed)
        torch.cuda.synchronize()
        assert torch.isfinite(ctx).all() and torch.isfinite(dqkv).all()
        out[fused] = (ctx, dqkv)
    for name, sl in (("ctx", None), ("dQ", slice(0, H)), ("dK", slice(H, 2 * H)), ("dV", slice(2 * H, 3 * H))):
        f = out[True][0] if sl is None else out[True][1][:, sl]
        u = out[False][0] if sl is None else out[False][1][:, sl]
        r = ref_ctx if sl is None else ref_dqkv[:, sl]
        ef, eu = rel(f, r), rel(u, r)
        print(f"B={B} L={L} p={p} {name}: fused {ef:.3e} unfused {eu:.3e}")
        assert ef <= 2e-2 and ef <= 1.25 * eu + 2e-3, (name, ef, eu)


def test_fused_attention_in_bert_step_matches_unfused(monkeypatch):
    """A whole bf16 text-only train step (BERT + head, dropout 0.1) with the fused kernels vs the unfused ones (same
    weights, inputs and dropout seeds): logits and every BERT parameter gradient within bf16 tolerance."""
    from vcg_hip import _lib, synth
    from vcg_hip.build import build_model
    from vcg_hip.functions import cross_entropy
    _lib.call("vcg_init", 0)
    _, ids, mask, labels = synth.clip_batch(4, 1, 8, 8, 128, seed=7, device=DEV)
    mask[1, 70:] = 0
    res = {}
    from vcg_hip.bert import BertEncoderEngine
    for flag in ("1", "0"):
        monkeypatch.setattr(BertEncoderEngine, "fused_attn", flag == "1")
        m = build_model("text", seed=7, device=DEV, precision="bf16", dropout=0.1).train()
        torch.manual_seed(11)  # the dropout seeds (vcg_hip.nn.new_seed) come from torch's RNG
        logits, _ = m(ids, mask)
        cross_entropy(logits, labels).backward()
        torch.cuda.synchronize()
        res[flag] = (logits.detach().float().cpu(),
                     {n: p.grad.detach().float().cpu().clone() for n, p in m.named_parameters() if p.grad is not None})
    l1, g1 = res["1"]
    l0, g0 = res["0"]
    assert (l1 - l0).abs().max().item() < 5e-2
    assert g1.keys() == g0.keys() and len(g1) > 100
    # the key bias gradient is zero in exact arithmetic (a row-constant score shift leaves the softmax unchanged):
    # both paths hold rounding noise there, compared by its size instead
    kb = [n for n in g1 if n.endswith("attention.self.key.bias")]
    assert len(kb) == 12
    for n in kb:
        ref = g1[n.replace("key.bias", "query.bias")].norm()
        assert g1[n].norm() < 5e-2 * ref and g0[n].norm() < 5e-2 * ref, (n, g1[n].norm(), g0[n].norm(), ref)
    errs = sorted((rel(g1[n], g0[n]), n) for n in g1 if n not in kb and g0[n].norm() > 0)
    print("grad rel errors: median %.3e, worst %s" % (errs[len(errs) // 2][0], errs[-3:]))
    assert errs[len(errs) // 2][0] < 3e-2 and errs[-1][0] < 1e-1


@pytest.mark.parametrize("p", [0.0, 0.1])
def test_varlen_attention_matches_padded(p):
    """Packed (unpadded) sequences (vcg_bert_attn_fwd/bwd_varlen, bert.Packing): the kept rows' ctx and dQ | dK | dV
    equal the padded kernels' bit for bit where the kept rows are a prefix of the padded ones (same key positions and
    dropout counters), given the dropped rows' upstream gradient is zero as in the model; a sequence with a masked hole
    matches within rounding without dropout; a sequence without any key keeps all its rows (uniform attention, as HF)."""
    from vcg_hip import _lib
    from vcg_hip.bert import Packing, attention_bwd, attention_fwd
    _lib.call("vcg_init", 0)
    B, L, nh, H = 5, 128, 12, 768
    Lp = L
    lens = [128, 77, 1, 50]
    mask_np = np.zeros((B, L), np.int64)
    for b, n in enumerate(lens):
        mask_np[b, :n] = 1
    mask_np[4, :10] = 1
    mask_np[4, 16:40] = 1                  # a hole: kept rows 0-9, 16-39 (positions shift when packed)
    mask_np[2, :] = 0                      # no key at all: every row kept
    pk = Packing(mask_np.copy(), DEV)
    rows = pk.rows.cpu()
    assert pk.R == 128 + 77 + 128 + 50 + 34
    g = torch.Generator().manual_seed(5)
    qkv = (torch.randn(B * L + 8, 3 * H, generator=g) * 1.5).to(torch.bfloat16)
    dctx = torch.randn(B * L, H, generator=g).to(torch.bfloat16)
    drop = torch.ones(B * L, dtype=torch.bool)
    drop[rows] = False
    dctx[drop] = 0
    seed = 0xABCDEF + int(p * 10)
    mask = torch.from_numpy(mask_np).to(DEV)
    ctx_p, att_p = attention_fwd(qkv.to(DEV), mask, B, nh, L, Lp, 64, 0.125, p, seed, True)
    dqkv_p = attention_bwd(qkv.to(DEV), dctx.to(DEV), ctx_p, mask, att_p, B, nh, L, Lp, 64, 0.125, p, seed)
    qkv_k = torch.cat([qkv[rows], torch.zeros(8, 3 * H, dtype=qkv.dtype)]).to(DEV)
    ctx_k, att_k = attention_fwd(qkv_k, pk.keys, B, nh, L, Lp, 64, 0.125, p, seed, True, seq=pk.seq, rows=pk.R)
    dqkv_k = attention_bwd(qkv_k, dctx[rows].to(DEV), ctx_k, pk.keys, att_k, B, nh, L, Lp, 64, 0.125, p, seed,
                           seq=pk.seq, rows=pk.R)
    torch.cuda.synchronize()
    ctx_p, dqkv_p, ctx_k, dqkv_k = (t.cpu() for t in (ctx_p, dqkv_p, ctx_k, dqkv_k))
    seq = pk.seq.cpu().tolist()
    for b in range(B):
        kr = rows[seq[b]:seq[b + 1]]
        a, c = slice(seq[b], seq[b + 1]), kr
        if b == 4:  # (with dropout its shifted key positions draw other dropout counters: another valid sample)
            if p == 0:
                assert rel(ctx_k[a], ctx_p[c]) < 5e-3 and rel(dqkv_k[a], dqkv_p[c]) < 5e-3, b
        else:
            assert torch.equal(ctx_k[a], ctx_p[c]) and torch.equal(dqkv_k[a], dqkv_p[c]), b


@pytest.mark.parametrize("case", ["prefix", "holes"])
def test_unpadded_bert_in_two_stream_step(monkeypatch, case):
    """A whole bf16 TwoStream train step (dropout 0) with BERT's padded rows dropped (BertEncoderEngine.unpad) and its
    last layer past the attention on the position-0 rows only (cls_last) vs every row computed: logits bit-identical (prefix masks: the kept rows see the padded computation exactly), every
    parameter gradient within fp32 summation-order rounding (the weight-gradient and bias sums run over fewer rows)."""
    from vcg_hip import _lib, synth
    from vcg_hip.bert import BertEncoderEngine, PackingRequest
    from vcg_hip.build import build_two_stream
    from vcg_hip.functions import cross_entropy
    _lib.call("vcg_init", 0)
    T, HW, L = 2, 64, 128
    frames, ids, mask, labels = synth.clip_batch(6, T, HW, HW, L, seed=21, device=DEV)
    assert (mask == 0).any()
    if case == "holes":  # masked positions inside the text, a masked CLS, a window without any key
        mask[0, 10:20] = 0
        mask[1, 0] = 0
        mask[2] = 0
    res = {}
    for unpad in (True, False):  # (the reference arm also runs the last layer on every row: cls_last off)
        monkeypatch.setattr(BertEncoderEngine, "unpad", unpad)
        monkeypatch.setattr(BertEncoderEngine, "cls_last", unpad)
        PackingRequest._last = PackingRequest._mirror = None
        m = build_two_stream(clip_frame_num=T, seed=5, device=DEV, precision="bf16", dropout=0.0).train()
        logits, _ = m(frames, ids, mask)
        cross_entropy(logits, labels).backward()
        torch.cuda.synchronize()
        res[unpad] = (logits.detach().float().cpu(),
                      {n: p.grad.detach().double().cpu().clone() for n, p in m.named_parameters() if p.grad is not None})
    (l1, g1), (l0, g0) = res[True], res[False]
    if case == "prefix":
        assert torch.equal(l1, l0)
    else:  # (shifted key positions: the same sums in another order)
        assert (l1 - l0).abs().max().item() < 2e-3
    assert g1.keys() == g0.keys()
    errs = sorted((rel(g1[n], g0[n]), n) for n in g1 if g0[n].norm() > 1e-3 * max(v.norm() for v in g0.values()))
    print(f"{case}: unpadded vs padded grad rel errors: median %.3e, worst %s" % (errs[len(errs) // 2][0], errs[-3:]))
    assert errs[-1][0] < (2e-3 if case == "prefix" else 5e-2), errs[-3:]
