"""BERT-base encoder on libvcg_hip (HF BertModel semantics, eager attention), forward and a
hand-written backward.

Reference use: TwoStream.forward -> lang_model(input_ids, attention_mask).pooler_output
(model/fusion/two_stream.py:172-179) with lang_model = BertModel('bert-base-uncased')
(model/lang/bert_hugface.py:20). Per layer: fused QKV GEMM -> attention (bf16, L <= 128: ONE fused
kernel per direction, bert_attn.hip, nothing L x L in HBM; otherwise batched QK^T -> masked softmax (+dropout) ->
batched PV) -> out-proj GEMM -> LN(dropout(.)+res) -> FFN1 GEMM with erf-GELU
epilogue -> FFN2 GEMM -> LN(dropout(.)+res); pooler = tanh(W h[:,0] + b).

Unpadded sequences (Packing, bf16 with the fused attention, callers that read only the pooler output -- TwoStream,
two_stream.py:178-179): a padded position (attention_mask 0) is a masked key, so no kept row ever reads it, and the
pooler reads only row 0; its rows are therefore dropped from every GEMM, LayerNorm and attention of the encoder (the
embedding LayerNorm still runs padded, then the kept rows are gathered; its gradient is scattered back with zeros at
the padded rows, which is what they receive in the padded computation). With prefix masks every kept row sees
exactly the padded computation (same attention key positions and dropout counters).
"""
import math
import weakref

import numpy as np
import torch

from . import ops


# BERT's Linear GEMMs run on the wide-tile engine (ops.ACT_FLAG_WIDE, csrc/igemm_wide.hip: bias, bias + GELU with the
# pre-activation, GELU' of the pre-activation, residual addend), whatever the batch; the flag is ignored in fp32
WIDE = ops.ACT_FLAG_WIDE

def _seed(base, layer, site):
    return (base * 0x9E3779B1 + layer * 7919 + site * 104729) & ((1 << 63) - 1)


def _uniform_p(mods, what):
    """The common dropout rate of training-mode nn.Dropout modules (0 for modules in eval mode)."""
    ps = {float(d.p) if d.training else 0.0 for d in mods}
    if len(ps) != 1:
        raise NotImplementedError(f"native BERT: {what} dropout modules with different rates {sorted(ps)}")
    return ps.pop()


class _LinearT:
    """bf16 W^T [in][out] of the encoder's Linear weights (QKV, attention output, FFN1, FFN2), the K-contiguous B operand
    of the backward's input-gradient GEMMs dX = dY W, written by ONE vcg_transpose_multi launch per weight generation
    (flat.generation moves with every optimizer step) instead of a transpose per GEMM (QKV, FFN1) or the generic
    engine's N-contiguous B path (attention output: 37 -> 24 us per layer)."""

    def __init__(self, model, flat, dtype):
        self.flat = flat
        self.gen = None
        srcs = []
        H = model.config.hidden_size
        for lyr in model.encoder.layer:
            at = lyr.attention
            srcs.append(flat.compute_contiguous([at.self.query.weight, at.self.key.weight, at.self.value.weight],
                                                (3 * H, H), dtype))
            for w in (at.output.dense.weight, lyr.intermediate.dense.weight, lyr.output.dense.weight):
                srcs.append(flat.compute_view(w, dtype))
        total = sum(s.numel() for s in srcs)
        dev = srcs[0].device
        self.buf = torch.empty(total, dtype=dtype, device=dev)
        self.t = {}
        desc, off, tiles = [], 0, 0
        for s in srcs:
            rows, cols = s.shape
            dst = self.buf[off:off + s.numel()].view(cols, rows)
            self.t[s.data_ptr()] = dst
            desc.append([s.data_ptr(), dst.data_ptr(), rows, cols, tiles])
            off += s.numel()
            tiles += ((rows + 63) // 64) * ((cols + 63) // 64)
        self.desc = torch.tensor(desc, dtype=torch.int64).to(dev)
        self.n, self.tiles = len(desc), tiles
        self.ptrs = [s.data_ptr() for s in srcs]

    def refresh(self):
        if self.gen != self.flat.generation:
            ops.transpose_multi(self.desc, self.n, self.tiles)
            self.gen = self.flat.generation

    def get(self, W):
        return self.t.get(W.data_ptr())


def pack_rows(mask_np):
    """Host side of Packing: (rows int64 [R] = flat b*L + t of the kept rows in order, seq int32 [B+1] prefix offsets,
    keys int64 [R] = the kept rows' mask values, cls int64 [B] = the packed row of each sequence's position 0)."""
    B, L = mask_np.shape
    keep = mask_np != 0
    keep[~keep.any(1)] = True
    keep[:, 0] = True
    seq = np.zeros(B + 1, dtype=np.int32)
    seq[1:] = np.cumsum(keep.sum(1))
    rows = np.flatnonzero(keep.reshape(-1)).astype(np.int64)
    return rows, seq, mask_np.reshape(-1)[rows].astype(np.int64), seq[:-1].astype(np.int64)


class Packing:
    """The kept rows of a padded [B, L] batch: every position with attention_mask != 0, plus position 0 (the pooler's
    row, even if masked), plus every row of a sequence without any key (HF then attends uniformly to all L rows).
    rows: flat b*L + t of the kept rows in order (int64 [R]); seq: int32 [B+1] prefix offsets; keys: the kept rows'
    mask values (int64 [R], the fused attention's key flags); cls: the packed row of each sequence's position 0."""

    def __init__(self, mask_np, device):
        B, L = mask_np.shape
        rows, seq, keys, cls = pack_rows(mask_np)
        self.B, self.L, self.R = B, L, int(seq[-1])
        host = [torch.from_numpy(a).pin_memory() for a in (rows, seq, keys, cls)]
        self.rows, self.seq, self.keys, self.cls = (t.to(device, non_blocking=True) for t in host)
        self._host = host  # (the pinned sources stay alive until the copies have run: the engine holds the Packing)


class PackingRequest:
    """The packing of a device attention mask: the host needs the mask, so a device-to-host copy is issued on the
    caller's stream (behind whatever produced the mask) and waited for in get(). The host copy is kept per base tensor
    (a mask that is a view -- long_video.score_windows' batches are slices of one mask of the whole video -- is read
    from its base's copy: one copy for all batches, no wait after the first), so a batch fed again, or the next slice
    of the same base, costs no device round trip while the base's version is unchanged."""
    _mirror = None  # (weakref to the base tensor, its _version, pinned host copy of the base)
    _last = None    # (weakref to the mask, its _version, its Packing)

    def __init__(self, mask):
        base = mask._base if mask._base is not None else mask
        self.mask, self.base, self.pk, self.ev = mask, base, None, None
        last = PackingRequest._last
        if last is not None and last[0]() is mask and last[1] == mask._version:
            self.pk = last[2]
            return
        mir = PackingRequest._mirror
        if mir is not None and mir[0]() is base and mir[1] == base._version:
            self.host = mir[2]
            return
        self.host = torch.empty(base.shape, dtype=base.dtype, pin_memory=True)
        self.host.copy_(base, non_blocking=True)
        self.ev = torch.cuda.Event()
        self.ev.record()

    def get(self):
        if self.pk is None:
            if self.ev is not None:
                self.ev.synchronize()
                PackingRequest._mirror = (weakref.ref(self.base), self.base._version, self.host)
                self.ev = None
            m, b = self.mask, self.base
            flat = self.host.reshape(-1).numpy()
            it = flat.itemsize
            view = np.lib.stride_tricks.as_strided(flat[m.storage_offset() - b.storage_offset():], shape=tuple(m.shape),
                                                   strides=tuple(st * it for st in m.stride()), writeable=False)
            self.pk = Packing(np.ascontiguousarray(view), m.device)
            PackingRequest._last = (weakref.ref(m), m._version, self.pk)
            self.mask = self.base = self.host = None
        return self.pk


class BertEncoderEngine:
    # bf16 L <= 128: the fused attention kernels (bert_attn.hip); False: the unfused kernels (tests compare both)
    fused_attn = True
    # unpadded sequences (Packing) where the caller reads only the pooler output and the fused attention applies;
    # False: every padded row is computed (tests compare both)
    unpad = True
    # bf16 backward: the Linear weight / bias gradients (split-K GEMMs + column sums) on a side stream, concurrently
    # with the input-gradient chain they branch off; False: one stream
    wgrad_stream = True
    # where only the pooler output is read: the last layer after its attention (output projection, LayerNorms, FFN)
    # runs on the B position-0 rows only -- the pooler reads nothing else (its K / V still cover every row)
    cls_last = True

    def __init__(self, model, flat, dtype):
        self.m = model
        self.flat = flat
        self.dtype = dtype
        self.wt = None
        self.pooled_only = False  # the caller reads only the pooler output (TwoStream): the rows may be unpadded
        self.packing = None  # forward()'s default packing (a Packing / PackingRequest the caller made)
        if dtype == torch.bfloat16 and flat is not None:
            wt = getattr(model, "_vcg_bert_wt", None)
            if wt is None or wt.flat is not flat:
                wt = _LinearT(model, flat, dtype)
                object.__setattr__(model, "_vcg_bert_wt", wt)
            self.wt = wt

    def _fused_attn(self, L, dh):
        # (the fp32 parity mode always runs unfused)
        return self.dtype == torch.bfloat16 and L <= 128 and dh == 64 and BertEncoderEngine.fused_attn

    def _w(self, p):
        return self.flat.compute_view(p, self.dtype)

    def _gemm_dx(self, A, W, M, N, K, f32_out=False, **kw):
        """A [M, K] @ W [K, N] (W = a Linear weight [out=K, in=N]: the input gradient). bf16 with a long K
        (QKV, FFN1 input gradients: K = 2304 / 3072, N = 768): W^T is materialised (tiled transpose) so the
        LDS-DMA GEMM reads both operands K-contiguous (measured 87 -> 61 us at K = 3072, 67 -> 53 us at
        K = 2304; no gain at K = 768, tools/bench_bert_gemm.py)."""
        # (FFN2's input gradient with the GELU' epilogue stays on the 128 x 128 engine, whose staged epilogue reads the
        # pre-activation as full rows: 71 vs 82 us on the wide engine, profiles/r06_bert_gemm.txt)
        if kw.get("act", ops.ACT_NONE) != ops.ACT_GELU_BWD:
            kw["act"] = kw.get("act", ops.ACT_NONE) | WIDE
        wt = self.wt.get(W) if self.wt is not None else None
        if f32_out:  # + the fp32 residual-gradient stream, written in fp32 (bf16: W^T is resident)
            kw["act"] |= ops.ACT_FLAG_F32_OUT
            return ops.gemm(A, wt, M, N, K, K, K, out=torch.empty((M, N), dtype=torch.float32, device=A.device),
                            ldc=N, **kw)
        if wt is not None:
            return ops.gemm(A, wt, M, N, K, K, K, **kw)
        if self.dtype == torch.bfloat16 and K >= 2 * N:
            return ops.gemm(A, ops.transpose(W), M, N, K, K, K, **kw)
        return ops.gemm(A, W, M, N, K, K, N, transB=True, **kw)

    def packs(self, ids):
        """forward() would run unpadded (a PackingRequest is worth making)."""
        cfg = self.m.config
        return (BertEncoderEngine.unpad and self.pooled_only and self.m.pooler is not None and ids.is_cuda
                and self._fused_attn(ids.shape[1], cfg.hidden_size // cfg.num_attention_heads))

    def forward(self, ids, mask, need_grad, seed, packing=None):
        """packing: a Packing or PackingRequest of `mask` (only where packs()); its kept rows are computed, and the
        second output (the last hidden state) is then empty."""
        m, dt, flat = self.m, self.dtype, self.flat
        if packing is None:
            packing = self.packing
        cfg = m.config
        B, L = ids.shape
        H = cfg.hidden_size
        nh = cfg.num_attention_heads
        dh = H // nh
        Lp = (L + 7) // 8 * 8
        if isinstance(packing, PackingRequest):
            packing = packing.get()
        if packing is not None and packing.R == B * L:  # nothing to drop
            packing = None
        rows = B * L if packing is None else packing.R
        # dropout rates from the nn.Dropout modules, as HF's BertModel applies them (a caller may change .p after
        # construction); hidden dropout sites share one rate, attention-probability sites another
        hid = [emb_d for emb_d in [m.embeddings.dropout] + [d for lyr in m.encoder.layer
                                                            for d in (lyr.attention.output.dropout, lyr.output.dropout)]]
        att = [lyr.attention.self.dropout for lyr in m.encoder.layer]
        p_h = _uniform_p(hid, "hidden")
        p_a = _uniform_p(att, "attention-probability")
        eps = cfg.layer_norm_eps
        scale = 1.0 / math.sqrt(dh)
        dev = ids.device
        ids = ids.contiguous()
        mask = mask.to(torch.int64).contiguous()
        if need_grad and self.wt is not None:
            self.wt.refresh()  # (read only by the backward; issued here, on BERT's stream, beside the trunk)

        lib = WIDE
        emb = m.embeddings
        h, e_mean, e_rstd = ops.embed_ln_fwd(ids, emb.word_embeddings.weight, emb.position_embeddings.weight,
                                             emb.token_type_embeddings.weight, emb.LayerNorm.weight,
                                             emb.LayerNorm.bias, B, L, H, eps, dt, p_h, _seed(seed, 0, 0))
        if packing is not None:
            h = h.index_select(0, packing.rows)
        att_mask, seq = (mask, None) if packing is None else (packing.keys, packing.seq)
        co = (BertEncoderEngine.cls_last and self.pooled_only and m.pooler is not None and self._fused_attn(L, dh))
        cls_idx = None
        if co:
            cls_idx = packing.cls if packing is not None else torch.arange(0, B * L, L, dtype=torch.int64, device=dev)
        nl = len(m.encoder.layer)
        saved_layers = []
        for i, layer in enumerate(m.encoder.layer):
            at = layer.attention
            sq, sk, sv = at.self.query, at.self.key, at.self.value
            Wqkv = flat.compute_contiguous([sq.weight, sk.weight, sv.weight], (3 * H, H), dt)
            bqkv = flat.contiguous_view([sq.bias, sk.bias, sv.bias], (3 * H,), "data")
            qkv_buf = torch.empty((rows + 8, 3 * H), dtype=dt, device=dev)  # +8 rows: padded key reads
            qkv = qkv_buf[:rows]
            ops.gemm(h, Wqkv, rows, 3 * H, H, H, H, out=qkv, ldc=3 * H, bias=bqkv, act=lib)
            sa = _seed(seed, i + 1, 1)
            ctx, att = attention_fwd(qkv_buf, att_mask, B, nh, L, Lp, dh, scale, p_a, sa, self._fused_attn(L, dh),
                                     seq=seq, rows=rows)
            lco = co and i == nl - 1  # (the last layer past its attention: the CLS rows only)
            hs, ctxs, lr = (h.index_select(0, cls_idx), ctx.index_select(0, cls_idx), B) if lco else (h, ctx, rows)
            ao = ops.gemm(ctxs, self._w(at.output.dense.weight), lr, H, H, H, H, bias=at.output.dense.bias, act=lib)
            s1 = _seed(seed, i + 1, 2)
            h1, m1, r1 = ops.ln_fwd(ao, hs, at.output.LayerNorm.weight, at.output.LayerNorm.bias, lr, H, eps, p_h, s1)
            inter, out = layer.intermediate.dense, layer.output.dense
            I = inter.out_features
            pre = torch.empty((lr, I), dtype=dt, device=dev) if need_grad else None
            ff = ops.gemm(h1, self._w(inter.weight), lr, I, H, H, H, bias=inter.bias, act=ops.ACT_GELU | lib, aux=pre)
            fo = ops.gemm(ff, self._w(out.weight), lr, H, I, I, I, bias=out.bias, act=lib)
            s2 = _seed(seed, i + 1, 3)
            h2, m2, r2 = ops.ln_fwd(fo, h1, layer.output.LayerNorm.weight, layer.output.LayerNorm.bias, lr, H, eps,
                                    p_h, s2)
            if need_grad:
                saved_layers.append(dict(h=h, hs=hs, qkv_buf=qkv_buf, att=att, ctxs=ctxs, ao=ao, h1=h1, pre=pre,
                                         ff=ff, fo=fo, m1=m1, r1=r1, m2=m2, r2=r2, sa=sa, s1=s1, s2=s2, lr=lr,
                                         lco=lco))
            h = h2
        pooled = None
        if co:  # (h is already the B position-0 rows)
            cls, lda = h, H
        else:
            cls = h if packing is None else h.index_select(0, packing.cls)  # (packed: the B position-0 rows)
            lda = L * H if packing is None else H
        if m.pooler is not None:
            pd = m.pooler.dense
            pooled = ops.gemm(cls, self._w(pd.weight), B, H, H, lda, H, bias=pd.bias, act=ops.ACT_TANH)
        saved = None
        if need_grad:
            saved = dict(ids=ids, mask=att_mask, seq=seq, packing=packing, co=co, cls_idx=cls_idx, layers=saved_layers,
                         e_mean=e_mean,
                         e_rstd=e_rstd, h_last=cls, lda=lda, pooled=pooled, B=B, L=L, Lp=Lp, H=H, nh=nh, dh=dh,
                         p_h=p_h, p_a=p_a, scale=scale, seed=seed)
        if packing is not None or co:
            h = h.new_empty((0, H))  # (the padded rows' / the last layer's hidden states were not all computed)
        return pooled, h, saved

    def backward(self, d_pooled, d_last, sv, hooks=None):
        m, dt, flat = self.m, self.dtype, self.flat
        B, L, Lp, H, nh, dh = sv["B"], sv["L"], sv["Lp"], sv["H"], sv["nh"], sv["dh"]
        packing, co, cls_idx = sv["packing"], sv["co"], sv["cls_idx"]
        rows = B * L if packing is None else packing.R
        if (packing is not None or co) and d_last is not None and d_last.numel():
            raise RuntimeError("BertEncoderEngine: the pooled-only forward has no last hidden state to differentiate")
        p_h, p_a, scale, seed = sv["p_h"], sv["p_a"], sv["scale"], sv["seed"]
        dev = sv["ids"].device
        side = _WSide(dev) if (BertEncoderEngine.wgrad_stream and dt == torch.bfloat16 and dev.type == "cuda") else None
        wg = side.run if side is not None else (lambda fn, *t: fn())
        # the residual-gradient stream (the gradient w.r.t. each LayerNorm output, summed over the skip and the next
        # layer's input gradient) stays fp32 between the LayerNorm backwards, as torch autocast keeps it (its
        # LayerNorm outputs are fp32): bf16 roundings of it compounded over 24 LayerNorms
        g32 = dt == torch.bfloat16 and self.wt is not None
        gd = torch.float32 if g32 else dt
        if d_last is not None and d_last.numel():
            dh_ = d_last.to(gd).contiguous().clone()
        else:  # (co: the last layer's output is the B position-0 rows)
            dh_ = torch.zeros((B if co else rows, H), dtype=gd, device=dev)
        if d_pooled is not None and m.pooler is not None:
            pd = m.pooler.dense
            dpp = ops.tanh_bwd(d_pooled.to(dt).contiguous(), sv["pooled"])
            h_last, lda = sv["h_last"], sv["lda"]
            if pd.weight.requires_grad:
                ops.gemm_splitk(dpp, h_last, pd.weight.grad, H, H, B, H, lda, transA=True, transB=True)
                ops.colsum(dpp, H, B, H, pd.bias.grad)
            # dh[b*L] += dpp @ Wp (B rows: an fp32 GEMM on the fp32 stream)
            dpw = (dpp.float(), pd.weight.data) if g32 else (dpp, self._w(pd.weight))
            if co:
                ops.gemm(dpw[0], dpw[1], B, H, H, H, H, transB=True, out=dh_, ldc=H, residual=dh_, ldr=H)
            elif packing is None:
                ops.gemm(dpw[0], dpw[1], B, H, H, H, H, transB=True, out=dh_, ldc=L * H, residual=dh_, ldr=L * H)
            else:  # (dh_ is zero: the CLS rows receive the product)
                dh_.index_copy_(0, packing.cls, ops.gemm(dpw[0], dpw[1], B, H, H, H, H, transB=True,
                                                         out=torch.empty((B, H), dtype=gd, device=dev)))
            if hooks is not None:
                hooks(list(m.pooler.parameters()))
        for i in reversed(range(len(sv["layers"]))):
            s = sv["layers"].pop()
            lr = s["lr"]  # (rows past the attention: B for the CLS-only last layer)
            layer = m.encoder.layer[i]
            at = layer.attention
            inter, out = layer.intermediate.dense, layer.output.dense
            I = inter.out_features
            ln2 = layer.output.LayerNorm
            dfo, dh1_res = ops.ln_bwd(dh_, s["fo"], s["h1"], ln2.weight, s["m2"], s["r2"], ln2.weight.grad,
                                      ln2.bias.grad, lr, H, p_h, s["s2"], bias_grad=out.bias.grad)
            wg(lambda: ops.gemm_splitk(dfo, s["ff"], out.weight.grad, H, I, lr, H, I, transA=True, transB=True),
               dfo, s["ff"])
            dpre = self._gemm_dx(dfo, self._w(out.weight), lr, I, H, act=ops.ACT_GELU_BWD, residual=s["pre"], ldr=I)
            del dfo
            def ffn1_w(dpre=dpre, h1=s["h1"]):
                ops.gemm_splitk(dpre, h1, inter.weight.grad, I, H, lr, I, H, transA=True, transB=True)
                ops.colsum(dpre, I, lr, I, inter.bias.grad)
            wg(ffn1_w, dpre, s["h1"])
            dh1 = self._gemm_dx(dpre, self._w(inter.weight), lr, H, I, f32_out=g32, residual=dh1_res, ldr=H)
            del dpre, dh1_res
            ln1 = at.output.LayerNorm
            od = at.output.dense
            dao, dh_res = ops.ln_bwd(dh1, s["ao"], s["hs"], ln1.weight, s["m1"], s["r1"], ln1.weight.grad,
                                     ln1.bias.grad, lr, H, p_h, s["s1"], bias_grad=od.bias.grad)
            wg(lambda: ops.gemm_splitk(dao, s["ctxs"], od.weight.grad, H, H, lr, H, H, transA=True, transB=True),
               dao, s["ctxs"])
            dctx = self._gemm_dx(dao, self._w(od.weight), lr, H, H)
            del dao
            if s["lco"]:  # back to every row: the attention's other rows (and the residual) receive zero
                dctx = torch.zeros((rows, H), dtype=dctx.dtype, device=dev).index_copy_(0, cls_idx, dctx)
                dh_res = torch.zeros((rows, H), dtype=dh_res.dtype, device=dev).index_copy_(0, cls_idx, dh_res)
            # ---- attention backward
            qkv_buf = s["qkv_buf"]
            dqkv = attention_bwd(qkv_buf, dctx, None, sv["mask"], s["att"], B, nh, L, Lp, dh, scale, p_a,
                                 s["sa"], seq=sv["seq"], rows=rows)
            del dctx
            sq, sk, svv = at.self.query, at.self.key, at.self.value
            if sq.weight.requires_grad:
                gW = flat.contiguous_view([sq.weight, sk.weight, svv.weight], (3 * H, H), "grad")
                gb = flat.contiguous_view([sq.bias, sk.bias, svv.bias], (3 * H,), "grad")
                def qkv_w(dqkv=dqkv, h=s["h"], gW=gW, gb=gb):
                    ops.gemm_splitk(dqkv, h, gW, 3 * H, H, rows, 3 * H, H, transA=True, transB=True)
                    ops.colsum(dqkv, 3 * H, rows, 3 * H, gb)
                wg(qkv_w, dqkv, s["h"])
            Wqkv = flat.compute_contiguous([sq.weight, sk.weight, svv.weight], (3 * H, H), dt)
            dh_ = self._gemm_dx(dqkv, Wqkv, rows, H, 3 * H, f32_out=g32, residual=dh_res, ldr=H)
            del dqkv, dh_res, s
            if hooks is not None:  # (after the layer's weight gradients: on their stream)
                if side is not None:
                    side.run(lambda: hooks(list(layer.parameters())))
                else:
                    hooks(list(layer.parameters()))
        emb = m.embeddings
        if packing is not None:  # back to the padded rows (zero gradient at the dropped ones)
            dpad = torch.zeros((B * L, H), dtype=dh_.dtype, device=dev)
            dh_ = dpad.index_copy_(0, packing.rows, dh_)
        ops.embed_ln_bwd(dh_, sv["ids"], emb.word_embeddings.weight, emb.position_embeddings.weight,
                         emb.token_type_embeddings.weight, emb.LayerNorm.weight, sv["e_mean"], sv["e_rstd"],
                         emb.word_embeddings.weight.grad, emb.position_embeddings.weight.grad,
                         emb.token_type_embeddings.weight.grad, emb.LayerNorm.weight.grad, emb.LayerNorm.bias.grad,
                         B, L, H, p_h, _seed(seed, 0, 0),
                         pad_idx=-1 if emb.word_embeddings.padding_idx is None else emb.word_embeddings.padding_idx)
        if hooks is not None:
            hooks(list(emb.parameters()))
        if side is not None:  # every weight gradient is complete on the caller's stream
            side.join()


class _WSide:
    """BERT's weight-gradient side stream (one per device): run(fn, *tensors) issues fn there after everything issued so
    far on the caller's stream and keeps `tensors` referenced until an event after fn has completed (as the trunk's
    ResNetTrunk._hold; record_stream's deferred frees grow the pool when the side stream trails); join() makes the
    caller's stream wait for it."""
    _streams = {}

    def __init__(self, dev):
        key = dev.index if dev.index is not None else torch.cuda.current_device()
        st = _WSide._streams.get(key)
        if st is None:
            st = _WSide._streams[key] = torch.cuda.Stream(device=dev)
        self.s, self.pending = st, []

    def run(self, fn, *tensors):
        self.s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(self.s):
            out = fn()
        ev = torch.cuda.Event()
        ev.record(self.s)
        self.pending.append((ev, tensors))
        while self.pending and self.pending[0][0].query():
            self.pending.pop(0)
        return out

    def join(self):
        torch.cuda.current_stream().wait_stream(self.s)
        self.pending.clear()


def attention_fwd(qkv_buf, mask, B, nh, L, Lp, dh, scale, p_a, seed, fused, seq=None, rows=None):
    """ctx [B*L, H] of HF BertSelfAttention (eager) from the fused projection qkv_buf [B*L (+8), 3H] and the
    key mask [B, L]; returns (ctx, saved-for-backward). fused: bert_attn.hip (bf16, L <= 128, dh = 64: one kernel,
    row statistics saved); else QK^T GEMM -> masked softmax (+dropout) -> PV GEMM with S, P, Pd in HBM.
    seq: packed sequences (Packing.seq; fused only), `rows` rows, mask = the packed rows' key flags."""
    H = nh * dh
    rows = B * L if rows is None else rows
    dt, dev = qkv_buf.dtype, qkv_buf.device
    ctx = torch.empty((rows, H), dtype=dt, device=dev)
    if fused:
        stats = torch.empty((B * nh * 128, 2), dtype=torch.float32, device=dev)
        ops.bert_attn_fwd(qkv_buf, mask, ctx, stats, B, nh, L, Lp, scale, p_a, seed, seq=seq)
        return ctx, dict(stats=stats)
    assert seq is None, "packed sequences need the fused attention"
    Z = B * nh
    S = torch.empty((Z, L, Lp), dtype=dt, device=dev)
    ops.gemm_batched(qkv_buf, qkv_buf[:, H:], S, L, Lp, dh, 3 * H, 3 * H, Lp, L * 3 * H, dh, L * 3 * H, dh,
                     nh * L * Lp, L * Lp, B, nh)
    Pm = torch.empty_like(S)
    Pd = torch.empty_like(S) if p_a > 0 else None
    ops.attn_softmax_fwd(S, mask, Pm, Pd, B, nh, L, Lp, scale, p_a, seed)
    del S
    Pv = Pd if Pd is not None else Pm
    ops.gemm_batched(Pv, qkv_buf[:, 2 * H:], ctx, L, dh, L, Lp, 3 * H, H, nh * L * Lp, L * Lp, L * 3 * H, dh,
                     L * H, dh, B, nh, transB=True)
    return ctx, dict(P=Pm, Pd=Pd)


def attention_bwd(qkv_buf, dctx, ctx, mask, att, B, nh, L, Lp, dh, scale, p_a, seed, seq=None, rows=None):
    """dqkv [B*L, 3H] (dQ | dK | dV) from dctx = d ctx, given attention_fwd's saved state."""
    H = nh * dh
    rows = B * L if rows is None else rows
    dt, dev = qkv_buf.dtype, qkv_buf.device
    dqkv = torch.empty((rows, 3 * H), dtype=dt, device=dev)
    if "stats" in att:
        ops.bert_attn_bwd(qkv_buf, dctx, ctx, mask, att["stats"], dqkv, B, nh, L, Lp, scale, p_a, seed, seq=seq)
        return dqkv
    Z = B * nh
    dPd = torch.empty((Z, L, Lp), dtype=dt, device=dev)
    ops.gemm_batched(dctx, qkv_buf[:, 2 * H:], dPd, L, Lp, dh, H, 3 * H, Lp, L * H, dh, L * 3 * H, dh,
                     nh * L * Lp, L * Lp, B, nh)
    Pv = att["Pd"] if att["Pd"] is not None else att["P"]
    # dV = Pd^T dO
    ops.gemm_batched(Pv, dctx, dqkv[:, 2 * H:], L, dh, L, Lp, H, 3 * H, nh * L * Lp, L * Lp, L * H, dh,
                     L * 3 * H, dh, B, nh, transA=True, transB=True)
    dS = torch.empty_like(dPd)
    ops.attn_softmax_bwd(dPd, att["P"], dS, Z, L, Lp, scale, p_a, seed)
    del dPd
    # dQ = dS K ; dK = dS^T Q
    ops.gemm_batched(dS, qkv_buf[:, H:], dqkv, L, dh, L, Lp, 3 * H, 3 * H, nh * L * Lp, L * Lp, L * 3 * H, dh,
                     L * 3 * H, dh, B, nh, transB=True)
    ops.gemm_batched(dS, qkv_buf, dqkv[:, H:], L, dh, L, Lp, 3 * H, 3 * H, nh * L * Lp, L * Lp, L * 3 * H, dh,
                     L * 3 * H, dh, B, nh, transA=True, transB=True)
    return dqkv
