"""Drop-in for reference model/fusion/stacked_window_self_attention.py (VideoChapterWindowAttention 6-95,
VideoChapterBlock 98-145, StackedVideoChapterAttention 148-223): same constructors, submodule and parameter
names (state dicts interchange) and initialisation rules; the forward runs as ONE libvcg_hip launch per batch
of windows (window_attn.hip: each workgroup keeps its window's residual stream and activations in LDS through
all 6 layers and the classifier).

Training mode runs vcg_hip/wtrain.py instead: the same blocks as native autograd Functions (GEMMs, LayerNorm,
dropout, the short-window attention core with window_pos_bias), forward and backward on libvcg_hip.
"""

import torch
from torch import nn

from vcg_hip.window import pack_window_weights, window_attn_fwd


class VideoChapterWindowAttention(nn.Module):
    """stacked_window_self_attention.py:6-95 (parameters, init)."""

    def __init__(self, hidden_size, num_attention_heads, window_size, dropout=0.1):
        super().__init__()
        if hidden_size % num_attention_heads != 0:
            raise ValueError(
                f"The hidden size {hidden_size} is not a multiple of the number of attention "
                f"heads {num_attention_heads}.")
        self.num_attention_heads = num_attention_heads
        self.attention_head_size = hidden_size // num_attention_heads
        self.all_head_size = hidden_size
        self.window_size = window_size
        self.query = nn.Linear(hidden_size, hidden_size)
        self.key = nn.Linear(hidden_size, hidden_size)
        self.value = nn.Linear(hidden_size, hidden_size)
        self.out_proj = nn.Linear(hidden_size, hidden_size)
        self.attention_dropout = nn.Dropout(dropout)
        self.position_encoding = nn.Linear(1, hidden_size)
        self.window_pos_bias = nn.Parameter(torch.zeros(1, num_attention_heads, 1, 2 * window_size + 1))
        # _init_weights order of :33-46 (RNG consumption order matters for seeded runs)
        for lin in (self.query, self.key, self.value, self.out_proj):
            nn.init.xavier_uniform_(lin.weight)
        for lin in (self.query, self.key, self.value, self.out_proj):
            nn.init.zeros_(lin.bias)
        nn.init.normal_(self.window_pos_bias, mean=0.0, std=0.02)
        nn.init.xavier_uniform_(self.position_encoding.weight)
        nn.init.zeros_(self.position_encoding.bias)


class VideoChapterBlock(nn.Module):
    """stacked_window_self_attention.py:98-145 (pre-LN block: attention, then the 4-Linear GELU FFN)."""

    def __init__(self, hidden_size, num_attention_heads, window_size, dropout=0.1):
        super().__init__()
        self.attention_norm = nn.LayerNorm(hidden_size)
        self.ffn_norm = nn.LayerNorm(hidden_size)
        self.attention = VideoChapterWindowAttention(hidden_size, num_attention_heads, window_size, dropout)
        h = hidden_size
        self.ffn = nn.Sequential(
            nn.Linear(h, 2 * h), nn.GELU(), nn.Dropout(dropout),
            nn.Linear(2 * h, 4 * h), nn.GELU(), nn.Dropout(dropout),
            nn.Linear(4 * h, 2 * h), nn.GELU(), nn.Dropout(dropout),
            nn.Linear(2 * h, h), nn.Dropout(dropout))
        for mod in self.ffn:
            if isinstance(mod, nn.Linear):
                nn.init.xavier_uniform_(mod.weight)
                nn.init.zeros_(mod.bias)


class StackedVideoChapterAttention(nn.Module):
    """stacked_window_self_attention.py:148-223. forward(fusion_emb [B, 2w+1, hidden], clip_info) ->
    (logits [B, 2], probs [B, 2]) for the middle (target) clip of each window."""

    def __init__(self, config):
        super().__init__()
        self.num_layers = 6
        self.hidden_size = config.hidden_size
        self.num_attention_heads = config.num_attention_heads
        self.window_size = config.window_size
        self.layers = nn.ModuleList([
            VideoChapterBlock(config.hidden_size, config.num_attention_heads, config.window_size,
                              config.attention_probs_dropout_prob) for _ in range(self.num_layers)])
        self.final_layer_norm = nn.LayerNorm(config.hidden_size)
        h = config.hidden_size
        layers = []
        for i, o in ((h, h), (h, h), (h, h // 2), (h // 2, h // 4)):
            layers += [nn.Linear(i, o), nn.LayerNorm(o), nn.GELU(), nn.Dropout(0.1)]
        self.classifier = nn.Sequential(*layers, nn.Linear(h // 4, 2))
        for mod in self.classifier:
            if isinstance(mod, nn.Linear):
                nn.init.xavier_uniform_(mod.weight)
                nn.init.zeros_(mod.bias)
        self._packed = None
        self._packed_key = None

    def packed_weights(self):
        """The packed f32 parameter buffer, rebuilt when any parameter changed (in-place versions) or moved."""
        params = list(self.parameters())
        key = tuple((p.data_ptr(), p._version) for p in params)
        if self._packed is None or key != self._packed_key:
            with torch.no_grad():
                self._packed = pack_window_weights(self)
            self._packed_key = key
        return self._packed

    def forward(self, fusion_emb, clip_info=None):
        if self.training:  # native forward + backward, vcg_hip/wtrain.py
            from vcg_hip import wtrain
            logits = wtrain.window_attention(self, fusion_emb.float().contiguous())
            return logits, wtrain.softmax_rows(logits)
        S, P = fusion_emb.shape[1], 2 * self.window_size + 1
        if S > P:  # the reference's window_pos_bias[..., :S] broadcast fails the same way
            raise RuntimeError(f"window of {S} clips exceeds 2 * window_size + 1 = {P} (window_pos_bias length)")
        return window_attn_fwd(fusion_emb.float().contiguous(), self.packed_weights(), self.hidden_size,
                               self.num_attention_heads, P)
