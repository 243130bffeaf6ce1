"""ChapterHead on libvcg_hip: two projection GEMMs with relu epilogues, then either the fused final
Linear / softmax kernel (head_type "mlp") or the per-window SelfAttention kernel (head_type "attn")
(reference model/fusion/two_stream.py:8-48, 51-95, 188-189)."""
import torch

from . import ops
from .nn import new_seed


class HeadEngine:
    def __init__(self, head, flat, dtype):
        self.h = head
        self.flat = flat
        self.dtype = dtype

    def _w(self, p):
        return self.flat.compute_view(p, self.dtype)

    def forward(self, lang, vis, need_grad):
        """lang: [B, Dl] (compute dtype); vis: [B*T, Dv] fp32. Returns logits, prob (fp32)."""
        hd, dt = self.h, self.dtype
        if hd.head_type not in ("mlp", "attn"):
            raise RuntimeError(f"Unknown head_type {hd.head_type}")
        B = lang.shape[0]
        T, hid = hd.segment_size, hd.hidden_size
        vis_t = vis if dt == torch.float32 else ops.cast_from_f32(vis.contiguous(), dt)
        lang = lang.contiguous()
        Dv, Dl = hd.vision_emb_size, hd.lang_emb_size
        Vout = ops.gemm(vis_t, self._w(hd.vision_proj_head.weight), B * T, hid, Dv, Dv, Dv, act=ops.ACT_RELU)
        Lout = ops.gemm(lang, self._w(hd.lang_proj_head.weight), B, hid, Dl, Dl, Dl, act=ops.ACT_RELU)
        saved = dict(vis_t=vis_t, lang=lang, Vout=Vout, Lout=Lout, B=B) if need_grad else None
        if hd.head_type == "attn":
            # SelfAttention over the T+1 fused tokens, output of token 0 (two_stream.py:31-48)
            at = hd.head
            p = at.attn_drop.p if at.training else 0.0
            seed = new_seed() if p > 0.0 else 0
            logits, prob, st = ops.head_attn_fwd(Vout, Lout, at.query, at.key, at.value, at.proj, B, T, hid,
                                                 at.n_head, p, seed)
            if saved is not None:
                saved.update(attn=st, p=p, seed=seed)
            return logits, prob, saved
        W, b = hd.head.weight, hd.head.bias
        logits, prob = ops.head_mlp_fwd(Vout, Lout, W, b, B, T, hid, W.shape[0])
        return logits, prob, saved

    def backward(self, dlogits, sv):
        hd, dt = self.h, self.dtype
        B = sv["B"]
        T, hid = hd.segment_size, hd.hidden_size
        Dv, Dl = hd.vision_emb_size, hd.lang_emb_size
        if hd.head_type == "attn":
            at = hd.head
            dV, dL = ops.head_attn_bwd(sv["attn"], at.query, at.key, at.value, at.proj, dlogits.contiguous(),
                                       sv["Vout"], sv["Lout"], B, T, hid, at.n_head, sv["p"], sv["seed"])
        else:
            W = hd.head.weight
            req = W.requires_grad
            dV, dL = ops.head_mlp_bwd(sv["Vout"], sv["Lout"], W, dlogits.contiguous(), W.grad if req else None,
                                      hd.head.bias.grad if req else None, B, T, hid, W.shape[0])
        vp, lp = hd.vision_proj_head.weight, hd.lang_proj_head.weight
        if vp.requires_grad:
            ops.gemm_splitk(dV, sv["vis_t"], vp.grad, hid, Dv, B * T, hid, Dv, transA=True, transB=True)
        dvis = ops.gemm(dV, self._w(vp), B * T, Dv, hid, hid, Dv, transB=True)
        if lp.requires_grad:
            ops.gemm_splitk(dL, sv["lang"], lp.grad, hid, Dl, B, hid, Dl, transA=True, transB=True)
        dlang = ops.gemm(dL, self._w(lp), B, Dl, hid, hid, Dl, transB=True)
        dvis32 = dvis if dt == torch.float32 else ops.cast_to_f32(dvis)
        return dlang, dvis32
