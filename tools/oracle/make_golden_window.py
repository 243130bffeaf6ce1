"""Goldens for the window transformer StackedVideoChapterAttention (reference
model/fusion/stacked_window_self_attention.py:148-223, configured as two_stream_window.TwoStream.build_chapter_head
does at :342-348: 16 heads, attention dropout 0.1), produced by running the REFERENCE module in this container
(only the .npz output is committed; the reference never travels).

tests/golden/window_attn.npz
  w{w}_emb / w{w}_logits / w{w}_probs : hidden 128, window_size w in (1, 2) -> S = 2w+1 clips, batch 4, eval
      (dropout inactive); weights from vcg_hip/synth.py by state-dict name with prefix "window_attn."; inputs
      from numpy's default_rng(11 + w).
  short_*: window_size 2 module fed S = 3 clips (the reference slices window_pos_bias[..., :S]).
  c1win_* / c1xattn_* / c1{self_attn,bilinear,multiplication}_*: the full window TwoStream at C1 shapes with
      head_type "mlp" / "cross_attn" / the other three (c1_window); c1pad_*: "mlp" with clip 0 of every window
      the zero padding clip (frames, ids and mask all 0).
usage: python tools/oracle/make_golden_window.py
"""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import make_golden as mg  # noqa: E402  (puts the reference on sys.path; loads vcg_hip/synth.py by path)
from model.fusion.stacked_window_self_attention import StackedVideoChapterAttention  # noqa: E402  (reference)

H, NH, B = 128, 16, 4


def build(w):
    cfg = type("Config", (), {"hidden_size": H, "num_attention_heads": NH, "attention_probs_dropout_prob": 0.1,
                              "window_size": w})
    m = StackedVideoChapterAttention(cfg)
    mg.synth.init_params(m, mg.SEED, prefix="window_attn.")
    return m.eval()


def c1_window(out, w=1, T=4, B=2, head_type="mlp", tag="c1win", pad_first=False):
    """The reference window TwoStream (two_stream_window.py:291-444, head_type "mlp") at C1 shapes: 2w+1 clips of
    T=4 frames 112^2 + 32 tokens, batch 2, eval with the calibrated running BN statistics of bn_running_stats.npz.
    Inputs: synth.clip_batch over B*(2w+1) clips (clip-major within each window)."""
    from model.fusion import two_stream_window as ref_win
    ref = mg.build_reference(T=T)  # lang / TSM vision models, initialised by name
    m = ref_win.TwoStream(ref.lang_model, ref.vision_model, 768, 2048, T, 128, w)
    m.build_chapter_head(output_size=2, head_type=head_type)
    mg.synth.init_params(m, mg.SEED)
    mg.synth.load_bn_stats(m, dict(np.load(os.path.join(mg.GOLD, "bn_running_stats.npz"))))
    m.eval()
    n = 2 * w + 1
    frames, ids, mask, _ = mg.synth.clip_batch(B * n, T, 112, 112, 32, seed=mg.SEED)
    frames = frames.view(B, n, T, 3, 112, 112)
    ids, mask = ids.view(B, n, 32), mask.view(B, n, 32)
    if pad_first:  # a window running off the video start: clip 0 is the zero padding of youtube_dataset.py:460-470
        frames[:, 0] = 0
        ids[:, 0] = 0
        mask[:, 0] = 0
    info = {"clip_start_frame": torch.zeros(B, n, dtype=torch.long), "total_frames": torch.full((B,), 100),
            "target_clip_idx": torch.full((B,), w), "total_num_clips": torch.full((B,), n)}
    with torch.no_grad():
        lg, pr = m(frames, ids, mask, info)
    out.update({f"{tag}_logits": lg.numpy(), f"{tag}_prob": pr.numpy()})


def main():
    out = {}
    for w in (1, 2):
        m = build(w)
        rng = np.random.default_rng(11 + w)
        emb = rng.standard_normal((B, 2 * w + 1, H)).astype(np.float32)
        with torch.no_grad():
            lg, pr = m(torch.from_numpy(emb), None)
        out.update({f"w{w}_emb": emb, f"w{w}_logits": lg.numpy(), f"w{w}_probs": pr.numpy()})
        if w == 2:
            short = emb[:, :3].copy()
            with torch.no_grad():
                lg, pr = m(torch.from_numpy(short), None)
            out.update({"short_emb": short, "short_logits": lg.numpy(), "short_probs": pr.numpy()})
    c1_window(out)
    c1_window(out, head_type="cross_attn", tag="c1xattn")
    for ht in ("self_attn", "bilinear", "multiplication"):
        c1_window(out, head_type=ht, tag=f"c1{ht}")
    c1_window(out, tag="c1pad", pad_first=True)
    np.savez_compressed(os.path.join(mg.GOLD, "window_attn.npz"), **out)
    print({k: v.shape for k, v in out.items()})


if __name__ == "__main__":
    main()
