"""Training goldens of the window model, produced by running the REFERENCE two_stream_window.TwoStream
(model/fusion/two_stream_window.py:291-444 with ChapterHead :134-288 and stacked_window_self_attention.py) in this
container -- only the .npz output is committed; the reference never travels.

tests/golden/window_train.npz, per head type ht in (mlp, cross_attn, self_attn, multiplication, bilinear):
  {ht}_loss, {ht}_logits : one step at C1 shapes (B=2 windows, window_size 1 -> 3 clips of T=4 frames 112^2 + 32
      tokens; labels [0, 1]): model.train() with every nn.Dropout at p=0 and the vision BatchNorms in eval mode on the
      calibrated running statistics of bn_running_stats.npz (a well-conditioned, deterministic step: the native
      bf16 / fp32 differences are then rounding, not batch-statistics chaos), F.cross_entropy, backward;
  {ht}_norm_names / {ht}_norms32 / {ht}_norms64 : every parameter's gradient norm, reference fp32 and the same
      reference model in fp64 (exact);
  {ht}_idx::{name} / {ht}_g32::{name} / {ht}_g64::{name} : sampled gradient elements of the head / window
      transformer / BERT pooler / trunk tensors in TRACK.
Weights: vcg_hip/synth.py by state-dict name (the GPU test regenerates them); inputs synth.clip_batch(6, ...).
usage: python tools/oracle/make_golden_window_train.py
"""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import make_golden as mg  # noqa: E402  (reference on sys.path, vcg_hip/synth.py by path)

TRACK = ["window_attn.layers.0.attention.window_pos_bias", "window_attn.layers.5.ffn.9.weight",
         "window_attn.layers.2.attention.query.weight", "window_attn.layers.0.attention.position_encoding.weight",
         "window_attn.classifier.16.weight", "window_attn.classifier.1.weight", "window_attn.final_layer_norm.bias",
         "fusion_head.lang_proj_heads.0.0.weight", "fusion_head.vision_proj_heads.1.4.weight",
         "fusion_head.vision_proj_heads.2.8.bias", "lang_model.pooler.dense.weight",
         "vision_model.layer4.2.conv3.weight", "vision_model.conv1.weight"]
HEAD_TRACK = {"mlp": ["fusion_head.head.1.0.weight", "fusion_head.head.0.8.weight"],
              "cross_attn": ["fusion_head.head.query_proj.weight", "fusion_head.head.key_proj.weight",
                             "fusion_head.head.frame_pos_encoding.weight", "fusion_head.head.lang_norm.weight"],
              "self_attn": ["fusion_head.head.query.weight", "fusion_head.head.proj.weight"],
              "multiplication": ["fusion_head.lang_expand_layers.1.4.weight", "fusion_head.head.2.0.weight"],
              "bilinear": ["fusion_head.bilinear_layers.1.weight", "fusion_head.bilinear_layers.0.bias",
                           "fusion_head.head.2.3.weight"]}
HEADS = ("mlp", "cross_attn", "self_attn", "multiplication", "bilinear")
T, B, W, L = 4, 2, 1, 32


def build(head_type, dtype):
    from model.fusion import two_stream_window as ref_win
    ref = mg.build_reference(T=T)
    m = ref_win.TwoStream(ref.lang_model, ref.vision_model, 768, 2048, T, 128, W)
    m.build_chapter_head(output_size=2, head_type=head_type)
    mg.synth.init_params(m, mg.SEED)
    mg.synth.load_bn_stats(m, dict(np.load(os.path.join(mg.GOLD, "bn_running_stats.npz"))))
    m = m.to(dtype)
    if dtype == torch.float64:
        # the reference builds its position scalars with .float() (fp32), which an fp64 Linear(1, H) rejects: the
        # exact run casts the SAME fp32 values to fp64 (instance override of get_relative_positions)
        for mod in m.modules():
            if hasattr(mod, "get_relative_positions"):
                orig = mod.get_relative_positions
                mod.get_relative_positions = (lambda f: (lambda n: f(n).double()))(orig)
    m.train()
    for mod in m.modules():
        if isinstance(mod, torch.nn.Dropout):
            mod.p = 0.0
        if isinstance(mod, torch.nn.BatchNorm2d):
            mod.eval()
    return m


def step(head_type, dtype):
    m = build(head_type, dtype)
    n = 2 * W + 1
    frames, ids, mask, _ = mg.synth.clip_batch(B * n, T, 112, 112, L, seed=mg.SEED)
    frames = frames.view(B, n, T, 3, 112, 112).to(dtype)
    ids, mask = ids.view(B, n, L), mask.view(B, n, L)
    info = {"clip_start_frame": torch.zeros(B, n, dtype=torch.long), "total_frames": torch.full((B,), 100),
            "target_clip_idx": torch.full((B,), W), "total_num_clips": torch.full((B,), n)}
    logits, _ = m(frames, ids, mask, info)
    loss = torch.nn.functional.cross_entropy(logits, torch.tensor([0, 1]))
    loss.backward()
    return m, loss.item(), logits.detach().double().numpy()


def main():
    """usage: make_golden_window_train.py [head_type ...] (default: all); existing entries of other heads are kept."""
    torch.set_num_threads(os.cpu_count() or 8)
    path = os.path.join(mg.GOLD, "window_train.npz")
    heads = sys.argv[1:] or HEADS
    out = dict(np.load(path, allow_pickle=False)) if os.path.exists(path) else {}
    for ht in heads:
        out = {k: v for k, v in out.items() if not k.startswith(ht + "_")}
        m32, l32, lg32 = step(ht, torch.float32)
        m64, l64, lg64 = step(ht, torch.float64)
        p32, p64 = dict(m32.named_parameters()), dict(m64.named_parameters())
        names = [n for n, p in p32.items() if p.grad is not None]
        out[f"{ht}_loss"] = np.array([l32, l64])
        out[f"{ht}_logits"] = np.stack([lg32, lg64])
        out[f"{ht}_norm_names"] = np.array(names)
        out[f"{ht}_norms32"] = np.array([p32[n].grad.double().norm().item() for n in names])
        out[f"{ht}_norms64"] = np.array([p64[n].grad.norm().item() for n in names])
        for n in TRACK + HEAD_TRACK[ht]:
            idx = mg.sample_idx(p32[n].numel())
            out[f"{ht}_idx::{n}"] = idx
            out[f"{ht}_g32::{n}"] = p32[n].grad.reshape(-1)[idx].double().numpy()
            out[f"{ht}_g64::{n}"] = p64[n].grad.reshape(-1)[idx].numpy()
        print(ht, "loss", l32, l64, "params with grads", len(names))
        del m32, m64
    np.savez_compressed(path, **out)


if __name__ == "__main__":
    main()
