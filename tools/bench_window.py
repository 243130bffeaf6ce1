"""Window transformer (vcg_window_attn_fwd) throughput: windows/s for B windows of 2w+1 clip embeddings
(hidden 128, 16 heads), HIP events around `iters` launches on the current stream, after warm-up.
usage: python tools/bench_window.py [B] [w] [iters]"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "video-chapter-generation_amd"), REPO]

import torch  # noqa: E402


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 512  # VCG_WINDOW_G=<g> fixes the windows per workgroup
    w = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    iters = int(sys.argv[3]) if len(sys.argv) > 3 else 50
    from model.fusion.stacked_window_self_attention import StackedVideoChapterAttention
    from vcg_hip import synth
    from vcg_hip.window import window_attn_fwd
    H, nh, S = 128, 16, 2 * w + 1
    cfg = type("Config", (), {"hidden_size": H, "num_attention_heads": nh, "attention_probs_dropout_prob": 0.1,
                              "window_size": w})
    m = StackedVideoChapterAttention(cfg).cuda().eval()
    synth.init_params(m, 123, prefix="window_attn.")
    packed = m.packed_weights()
    emb = torch.randn(B, S, H, device="cuda")
    for _ in range(5):
        window_attn_fwd(emb, packed, H, nh, S)
    torch.cuda.synchronize()
    t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0.record()
    for _ in range(iters):
        window_attn_fwd(emb, packed, H, nh, S)
    t1.record()
    torch.cuda.synchronize()
    ms = t0.elapsed_time(t1) / iters
    flop = 6 * 2 * S * 24 * H * H + 2 * (3 * H * H + H * H // 2 + H * H // 8)  # blocks + classifier (per window)
    print(json.dumps({"kernel": "window_attn_fwd_kernel", "windows": B, "G": os.environ.get("VCG_WINDOW_G", "auto"), "clips_per_window": S, "hidden": H,
                      "ms_per_launch": round(ms, 4), "windows_per_s": round(B / ms * 1e3, 1),
                      "gflop_per_s": round(flop * B / ms / 1e6, 1),
                      "weight_bytes_per_window_from_L2": packed.numel() * 4}))


if __name__ == "__main__":
    main()
