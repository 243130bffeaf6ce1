"""Window model inference throughput (reference two_stream_window.TwoStream, eval): B windows of 2w+1 clips, each
clip 16 x 224^2 frames + 128 tokens; per clip the native BERT + TSM-ResNet-50 engines and the window ChapterHead,
then one window-transformer launch. Synthetic seeded inputs in HBM, random-init weights; HIP events over `iters`
forwards after one warm-up. The trunk / BERT run in `--precision` (bf16 default), the heads in fp32.
usage: python tools/bench_window_model.py [--batch 16] [--window 1] [--head mlp] [--iters 3] [--precision bf16]"""
import argparse
import contextlib
import io
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "video-chapter-generation_amd"), REPO]

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--window", type=int, default=1)
    ap.add_argument("--head", default="mlp")
    ap.add_argument("--iters", type=int, default=3)
    ap.add_argument("--precision", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--frames", type=int, default=16)
    ap.add_argument("--res", type=int, default=224)
    ap.add_argument("--tokens", type=int, default=128)
    ap.add_argument("--cached", action="store_true", help="score all `batch` clips of a video as targets from "
                    "per-clip embeddings (each clip's BERT / trunk pass once, TwoStream.forward_embeddings)")
    a = ap.parse_args()
    from model.fusion.two_stream_window import TwoStream
    from model.lang.bert_hugface import BertHugface
    from model.vision.resnet50_tsm import Resnet50TSM
    from vcg_hip import synth
    from vcg_hip.nn import BertConfig
    B, n, T, R, L = a.batch, 2 * a.window + 1, a.frames, a.res, a.tokens
    with contextlib.redirect_stdout(io.StringIO()):
        lang = BertHugface(pretrain_stage=False, config=BertConfig())
    vis = Resnet50TSM(segments_size=T, shift_div=8, pretrain_stage=False)
    m = TwoStream(lang.base_model, vis.base_model, 768, 2048, T, 128, a.window)
    with contextlib.redirect_stdout(io.StringIO()):
        m.build_chapter_head(output_size=2, head_type=a.head)
    m = m.cuda().eval()
    synth.init_params(m, 123)
    m.lang_model.precision = m.vision_model.precision = a.precision
    if a.cached:
        return cached(m, a, B, n, T, R, L)
    frames, ids, mask, _ = synth.clip_batch(B * n, T, R, R, L, seed=123, device="cuda")
    frames = frames.view(B, n, T, 3, R, R)
    ids, mask = ids.view(B, n, L), mask.view(B, n, L)
    with torch.no_grad():
        m(frames, ids, mask, None)
        torch.cuda.synchronize()
        t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0.record()
        for _ in range(a.iters):
            lg, pr = m(frames, ids, mask, None)
        t1.record()
        torch.cuda.synchronize()
    ms = t0.elapsed_time(t1) / a.iters
    print(json.dumps({"model": "window TwoStream (eval)", "head_type": a.head, "windows": B, "clips_per_window": n,
                      "frames": T, "res": R, "tokens": L, "precision": a.precision, "ms_per_batch": round(ms, 2),
                      "windows_per_s": round(B / ms * 1e3, 1), "clips_per_s": round(B * n / ms * 1e3, 1),
                      "finite": bool(torch.isfinite(lg).all().item())}))


def cached(m, a, V, n, T, R, L):
    """A video of V clips, every clip a window target (window_clip_indices, -1 = zero padding clip): embeddings of
    the V clips + the zero clip once, then V windows from them."""
    from data.clip_windows import window_clip_indices
    from vcg_hip import synth
    frames, ids, mask, _ = synth.clip_batch(V + 1, T, R, R, L, seed=123, device="cuda")
    frames[V].zero_()
    ids[V].zero_()
    mask[V].zero_()
    win = torch.tensor([window_clip_indices(t, V, T, a.window) for t in range(V)], device="cuda")

    def run():
        lang, vis = m.clip_embeddings(frames, ids, mask)
        return m.forward_embeddings(lang[:V], vis[:V], win, lang[V], vis[V])
    with torch.no_grad():
        run()
        torch.cuda.synchronize()
        t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0.record()
        for _ in range(a.iters):
            lg, _ = run()
        t1.record()
        torch.cuda.synchronize()
    ms = t0.elapsed_time(t1) / a.iters
    print(json.dumps({"model": "window TwoStream (eval, per-clip embeddings cached)", "head_type": a.head,
                      "windows": V, "clips_per_window": n, "clip_passes": V + 1, "frames": T, "res": R, "tokens": L,
                      "precision": a.precision, "ms_per_video": round(ms, 2), "windows_per_s": round(V / ms * 1e3, 1),
                      "finite": bool(torch.isfinite(lg).all().item())}))


if __name__ == "__main__":
    main()
