"""Drop-in for reference model/fusion/two_stream_window.py (CrossAttention 11-91, SelfAttention 93-131,
ChapterHead 134-288, TwoStream 291-444): the window model that scores the middle clip of 2w+1 consecutive
clips. Same constructors, submodule / parameter names and head types; inference runs on libvcg_hip:

  per clip i:  BERT pooler (native BertModel), TSM-ResNet-50 trunk (native ResNet50 engine),
               ChapterHead(window_idx=i): the Linear -> LayerNorm -> ReLU chains as fp32 GEMMs with fused
               bias/activation epilogues + one LayerNorm/activation row kernel (vcg_hip/window.py mlp_chain)
  window:      StackedVideoChapterAttention over the stacked [B, 2w+1, hidden] fusion embeddings
               (one window_attn.hip launch).

Native scope: eval-mode forward of every head type: "mlp" (train_video_segment_update_accumulate.py:360's default),
"cross_attn" (test_video_segment_update.py:43's default; one cross_attn_fwd_kernel launch per clip), "self_attn"
(head_attn.hip's SelfAttention kernel, output_size = hidden), "bilinear" (x2 A^T on the GEMM path + a row-dot
kernel), "multiplication" (elementwise kernel).
Training (model.train()): forward and backward of "mlp", "cross_attn" (train_video_segment_ddp.py:579's default),
"self_attn", "multiplication" and "bilinear" (wtrain.BilinearFn: vcg_rowdot_fwd / _bwd + GEMMs) through
vcg_hip/wtrain.py (every op a libvcg_hip kernel pair: GEMMs, LayerNorm +
activation + dropout, the short-window attention core, position encodings), the per-clip BERT / trunk passes
through the native engines with the model's flat parameter / gradient buffers (TwoStream is the NativeRoot), and
the reference's AdamW grouping on the fused optimizer. No CPU / eager path.
"""
import math

import torch
from torch import nn
from einops import rearrange

from vcg_hip import wtrain
from vcg_hip.nn import NativeRoot, new_seed
from vcg_hip.optim import configure_adamw
from vcg_hip.window import bilinear, cross_attn_fwd, linear, mlp_chain, mul, pack_cross_attn_weights

from .stacked_window_self_attention import StackedVideoChapterAttention


class CrossAttention(nn.Module):
    """two_stream_window.py:11-91 (parameters and their _init_weights :38-48; the forward is a kernel:
    cross_attn_fwd in eval, vcg_hip/wtrain.cross_attention in training)."""

    def __init__(self, hidden_size, num_heads, dropout=0.1):
        super().__init__()
        if hidden_size % num_heads != 0:
            raise ValueError(f"The hidden size {hidden_size} is not a multiple of the number of attention "
                             f"heads {num_heads}.")
        self.hidden_size, self.num_heads, self.head_dim = hidden_size, num_heads, hidden_size // num_heads
        self.query_proj = nn.Linear(hidden_size, hidden_size)
        self.key_proj = nn.Linear(hidden_size, hidden_size)
        self.value_proj = nn.Linear(hidden_size, hidden_size)
        self.out_proj = nn.Linear(hidden_size, hidden_size)
        self.lang_norm = nn.LayerNorm(hidden_size)
        self.vision_norm = nn.LayerNorm(hidden_size)
        self.attention_dropout = nn.Dropout(dropout)
        self.output_dropout = nn.Dropout(dropout)
        self.frame_pos_encoding = nn.Linear(1, hidden_size)
        scale = 1.0 / math.sqrt(self.head_dim)  # _init_weights (:38-48), in the reference's RNG order
        for proj in (self.query_proj, self.key_proj, self.value_proj, self.out_proj):
            nn.init.xavier_uniform_(proj.weight, gain=scale)
            nn.init.zeros_(proj.bias)
        nn.init.xavier_uniform_(self.frame_pos_encoding.weight)
        nn.init.zeros_(self.frame_pos_encoding.bias)


class SelfAttention(nn.Module):
    """two_stream_window.py:93-131 (parameters only)."""

    def __init__(self, n_embd, n_head, output_size, attn_pdrop=0.1, resid_pdrop=0.1):
        super().__init__()
        assert n_embd % n_head == 0
        self.n_head, self.n_embd = n_head, n_embd
        self.key = nn.Linear(n_embd, n_embd)
        self.query = nn.Linear(n_embd, n_embd)
        self.value = nn.Linear(n_embd, n_embd)
        self.attn_drop = nn.Dropout(attn_pdrop)
        self.resid_drop = nn.Dropout(resid_pdrop)
        self.proj = nn.Linear(n_embd, output_size)


def _proj(i, h1, h2, o):
    """Linear(i, h1) LN ReLU Dropout Linear(h1, h2) LN ReLU Dropout Linear(h2, o) (the per-clip projections)."""
    return nn.Sequential(nn.Linear(i, h1), nn.LayerNorm(h1), nn.ReLU(), nn.Dropout(0.1),
                         nn.Linear(h1, h2), nn.LayerNorm(h2), nn.ReLU(), nn.Dropout(0.1), nn.Linear(h2, o))


class ChapterHead(nn.Module):
    """two_stream_window.py:134-288: per-clip (window_idx) projection heads and fusion head."""

    def __init__(self, lang_emb_size, vision_emb_size, segment_size, hidden_size, window_size, output_size,
                 head_type="mlp"):
        super().__init__()
        self.lang_emb_size, self.vision_emb_size = lang_emb_size, vision_emb_size
        self.segment_size, self.hidden_size, self.head_type = segment_size, hidden_size, head_type
        self.window_size = window_size
        self.num_clips = n = 2 * window_size + 1
        h = hidden_size
        self.lang_proj_heads = nn.ModuleList([
            nn.Sequential(nn.Linear(lang_emb_size, lang_emb_size // 2), nn.LayerNorm(lang_emb_size // 2), nn.ReLU(),
                          nn.Dropout(0.1), nn.Linear(lang_emb_size // 2, h)) for _ in range(n)])
        self.vision_proj_heads = nn.ModuleList([_proj(vision_emb_size, 8 * h, 4 * h, h) for _ in range(n)])
        if head_type == "mlp":
            self.head = nn.ModuleList([_proj((segment_size + 1) * h, 8 * h, 4 * h, h) for _ in range(n)])
        elif head_type == "bilinear":
            self.bilinear_layers = nn.ModuleList([nn.Bilinear(h, h * segment_size, h * 2) for _ in range(n)])
            self.head = nn.ModuleList([
                nn.Sequential(nn.LayerNorm(h * 2), nn.ReLU(), nn.Dropout(0.1), nn.Linear(h * 2, h), nn.LayerNorm(h),
                              nn.ReLU(), nn.Dropout(0.1), nn.Linear(h, h)) for _ in range(n)])
        elif head_type == "multiplication":
            self.lang_expand_layers = nn.ModuleList([
                nn.Sequential(nn.Linear(h, h * 8), nn.LayerNorm(h * 8), nn.ReLU(), nn.Dropout(0.1),
                              nn.Linear(h * 8, h * segment_size), nn.LayerNorm(h * segment_size), nn.ReLU(),
                              nn.Dropout(0.1)) for _ in range(n)])
            self.head = nn.ModuleList([_proj(h * segment_size, 8 * h, 4 * h, h) for _ in range(n)])
        elif head_type == "self_attn":
            self.head = SelfAttention(h, 4, h)
        elif head_type == "cross_attn":
            self.head = CrossAttention(h, num_heads=16)
            self.output_proj = nn.Linear(h, output_size)
        else:
            raise RuntimeError(f"Unknown head_type {head_type}")

    def forward(self, lang_emb, vision_emb, window_idx):
        """lang_emb [B, lang_emb_size], vision_emb [B, segment_size, vision_emb_size] (f32) -> [B, hidden]."""
        from vcg_hip.ops import ACT_RELU, head_attn_fwd
        if self.training:
            return wtrain.chapter_head(self, lang_emb, vision_emb, window_idx)
        B = lang_emb.shape[0]
        lp, vp = self.lang_proj_heads[window_idx], self.vision_proj_heads[window_idx]
        lang_out = linear(mlp_chain(lang_emb.float().contiguous(), lp[:-1]), lp[-1], ACT_RELU)  # :262-263
        vis = vision_emb.reshape(-1, self.vision_emb_size).float().contiguous()
        vision_out = linear(mlp_chain(vis, vp[:-1]), vp[-1], ACT_RELU)                           # :265-267
        if self.head_type == "cross_attn":  # :284-286 (output_proj's result is unused by the reference)
            return cross_attn_fwd(lang_out, vision_out.view(B, self.segment_size, self.hidden_size),
                                  self._cross_weights(), self.hidden_size, self.head.num_heads)
        T, h = self.segment_size, self.hidden_size
        if self.head_type == "self_attn":  # :280-282: SelfAttention over cat([vision, lang]), token 0 -> proj
            at = self.head
            return head_attn_fwd(vision_out, lang_out, at.query, at.key, at.value, at.proj, B, T, h, at.n_head)[0]
        if self.head_type == "bilinear":  # :271-273
            fusion = bilinear(lang_out, vision_out.view(B, T * h), self.bilinear_layers[window_idx])
            return mlp_chain(fusion, self.head[window_idx])
        if self.head_type == "multiplication":  # :275-279
            expanded = mlp_chain(lang_out, self.lang_expand_layers[window_idx])
            return mlp_chain(mul(vision_out.view(B, T * h), expanded), self.head[window_idx])
        fusion = torch.cat([vision_out.view(B, T, h), lang_out.unsqueeze(1)], 1)
        return mlp_chain(fusion.view(B, -1), self.head[window_idx])                                 # :269-272

    def _cross_weights(self):
        key = tuple((p.data_ptr(), p._version) for p in self.head.parameters())
        if getattr(self, "_xkey", None) != key:
            with torch.no_grad():
                self._xpacked = pack_cross_attn_weights(self.head)
            self._xkey = key
        return self._xpacked


class _ClipCountingHooks:
    """Forwards a parameter group to the DDP hooks at its n-th report: the per-clip BERT / trunk backwards (any
    order) each report every group once, and the shared gradients are final after the last of the n clips."""

    def __init__(self, hooks, n):
        self.hooks, self.n, self.seen = hooks, n, {}

    def __call__(self, params):
        if isinstance(params, str) or not params:
            return
        key = tuple(id(p) for p in params)
        c = self.seen.get(key, 0) + 1
        self.seen[key] = c
        if c == self.n:
            self.hooks(params)


class TwoStream(NativeRoot, nn.Module):
    """two_stream_window.py:291-444. forward(img_clips [B, 2w+1, T, 3, H, W], text_ids [B, 2w+1, L],
    attention_masks [B, 2w+1, L], clip_info) -> (logits [B, 2], prob [B, 2]) of each window's middle clip."""

    def __init__(self, lang_model, vision_model, lang_embed_size, vision_embed_size, segment_size, hidden_size,
                 window_size):
        super().__init__()
        from model.fusion.two_stream import adopt_lang_model, adopt_vision_model
        self.lang_model = adopt_lang_model(lang_model)      # foreign (reference-built) encoders are converted
        self.vision_model = adopt_vision_model(vision_model)
        self.segment_size = segment_size
        self.lang_embed_size = lang_embed_size
        self.vision_embed_size = vision_embed_size
        self.hidden_size = hidden_size
        self.window_size = window_size
        h, layers, d = hidden_size, [], hidden_size * (2 * window_size + 1)
        for o in (h, h // 2, h // 4, h // 8, h // 16):  # window_mlp (:303-331; unused by the forward, kept for
            layers += [nn.Linear(d, o), nn.LayerNorm(o), nn.ReLU(), nn.Dropout(0.1)]  # state-dict parity)
            d = o
        self.window_mlp = nn.Sequential(*layers, nn.Linear(h // 16, 2))

    def build_chapter_head(self, output_size, head_type="mlp"):
        self.fusion_head = ChapterHead(self.lang_embed_size, self.vision_embed_size, self.segment_size,
                                       self.hidden_size, self.window_size, output_size, head_type)
        cfg = type("Config", (), {"hidden_size": self.hidden_size, "num_attention_heads": 16,
                                  "attention_probs_dropout_prob": 0.1, "window_size": self.window_size})
        self.window_attn = StackedVideoChapterAttention(cfg)

    def configure_optimizers(self, train_config):
        """AdamW with the reference's decay grouping (:355-388), as one fused kernel over the flat buffers."""
        return configure_adamw(self, train_config)

    def set_grad_hooks(self, hooks):
        """hooks(params) is called from the backward as parameter groups become final (DDP bucket all-reduce,
        vcg_hip/ddp.py). BERT and the trunk run once per window clip and share their parameters, so a group is
        final at its (2w+1)-th report (_ClipCountingHooks); the heads' gradients are reduced by the reducer's
        finish()."""
        object.__setattr__(self, "_vcg_hooks", hooks)

    def forward(self, img_clips, text_ids, attention_masks, clip_info=None):
        if self.training:
            return self._train_forward(img_clips, text_ids, attention_masks)
        B, n_clips, _ = text_ids.shape
        embs = []
        for i in range(n_clips):  # :395-433
            lang_emb = self.lang_model(input_ids=text_ids[:, i, :].contiguous(),
                                       attention_mask=attention_masks[:, i, :].contiguous()).pooler_output
            img = rearrange(img_clips[:, i], "b t c h w -> (b t) c h w").contiguous()
            vision_emb = self.vision_model(img).view(B, self.segment_size, -1)
            embs.append(self.fusion_head(lang_emb, vision_emb, i))
        return self.window_attn(torch.stack(embs, 1).contiguous(), clip_info)  # :435-444

    def _train_forward(self, img_clips, text_ids, attention_masks):
        """Training (and train-mode) forward, :390-444: per clip i BERT (pooler) and the TSM trunk run as native
        autograd Functions over the root's flat buffers (BatchNorm statistics of clip i's B*T frames, as the
        reference's per-clip vision_model call), then ChapterHead(window_idx=i) and the window transformer through
        vcg_hip/wtrain.py."""
        from vcg_hip.bert import BertEncoderEngine
        from vcg_hip.functions import BertFn, TrunkFn
        from vcg_hip.trunk import ResNetTrunk
        B, n_clips, _ = text_ids.shape
        f = self.native_flat()
        dt = self.compute_dtype()
        need_grad = torch.is_grad_enabled()
        dev = img_clips.device
        anchor = self._anchor(dev)
        embs = []
        hooks = getattr(self, "_vcg_hooks", None)
        counted = _ClipCountingHooks(hooks, n_clips) if (hooks is not None and need_grad) else None
        for i in range(n_clips):
            if self.vision_model.training:
                self._bump_bn_counters()  # every BatchNorm forward of the reference counts once per clip
            lang_emb, _ = BertFn.apply(text_ids[:, i, :].contiguous(), attention_masks[:, i, :].contiguous(), anchor,
                                       BertEncoderEngine(self.lang_model, f, dt), need_grad, new_seed(), counted)
            img = rearrange(img_clips[:, i], "b t c h w -> (b t) c h w").float().contiguous()
            vision_emb = TrunkFn.apply(img, anchor, ResNetTrunk(self.vision_model, dt), need_grad, counted)
            embs.append(self.fusion_head(lang_emb, vision_emb.view(B, self.segment_size, -1), i))
        return self.window_attn(torch.stack(embs, 1).contiguous(), None)

    # ---- long-video scoring from per-clip embeddings (not in the reference: a clip belongs to 2w+1 windows, so
    # ---- scoring every window with forward() runs its BERT / trunk pass 2w+1 times)
    def clip_embeddings(self, frames, text_ids, attention_mask, chunk=64):
        """Per-clip (lang_emb [N, 768], vision_emb [N, T, 2048]) f32 for N clips (frames [N, T, 3, H, W], ids / mask
        [N, L]), computed once per clip in chunks of `chunk` clips."""
        if self.training:
            raise RuntimeError("clip_embeddings is an inference helper: call model.eval() first")
        langs, viss = [], []
        for c0 in range(0, frames.shape[0], chunk):
            f = frames[c0:c0 + chunk]
            n = f.shape[0]
            langs.append(self.lang_model(input_ids=text_ids[c0:c0 + chunk].contiguous(),
                                         attention_mask=attention_mask[c0:c0 + chunk].contiguous()).pooler_output.float())
            img = rearrange(f, "b t c h w -> (b t) c h w").contiguous()
            viss.append(self.vision_model(img).float().view(n, self.segment_size, -1))
        return torch.cat(langs), torch.cat(viss)

    def forward_embeddings(self, lang_embs, vision_embs, window_indices, pad_lang=None, pad_vision=None):
        """Score windows from per-clip embeddings: window_indices [B, 2w+1] int64 clip rows (-1 = the zero padding
        clip, whose embeddings pad_lang [768] / pad_vision [T, 2048] are clip_embeddings() of an all-zero clip).
        Same result as forward() on the materialised windows; each clip's BERT / trunk pass runs once."""
        if self.training:
            raise RuntimeError("forward_embeddings is an inference helper: call model.eval() first")
        idx = window_indices.to(lang_embs.device).long()
        if bool((idx < 0).any()):
            if pad_lang is None or pad_vision is None:
                raise RuntimeError("window_indices hold padding (-1) clips: pass pad_lang / pad_vision")
            lang_embs = torch.cat([lang_embs, pad_lang.reshape(1, -1).float()])
            vision_embs = torch.cat([vision_embs, pad_vision.reshape(1, *vision_embs.shape[1:]).float()])
            idx = torch.where(idx < 0, torch.full_like(idx, lang_embs.shape[0] - 1), idx)
        embs = [self.fusion_head(lang_embs.index_select(0, idx[:, i]).contiguous(),
                                 vision_embs.index_select(0, idx[:, i]).contiguous(), i) for i in range(idx.shape[1])]
        return self.window_attn(torch.stack(embs, 1).contiguous(), None)
