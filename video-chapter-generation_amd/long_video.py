"""Long-video chapter-boundary inference on one MI355X (BASELINE config 5).

One decoded video (u8 frames [F, H, W, 3], 1 fps, resident in HBM) is scored end to end:
  1. sliding windows [s, s + T) for s in range(0, F - T, stride)  (the reference uses stride 2*max_offset = 4 s,
     `youtube_dataset.py:94`, `flat_video2clip_for_quick_infer.py:66`; config 5 asks for stride 1 s);
  2. each window's frames are gathered by the reference's frame-index rule (+2 away from the video ends,
     `youtube_dataset.py:180-190`, data/clip_windows.py:frame_index_table) and normalised as
     ToTensor + Normalize (`train_video_segment_point.py:383-386`) on the GPU straight into the stem's NHWC
     layout (ops.window_frames_u8) -- no host decode / upload per window;
  3. subtitles in (s - 1, e + 1) are tokenised as "[CLS] " + text, truncated / padded to L
     (`youtube_dataset.py:141-174`);
  4. TwoStream scores the windows in batches of consecutive windows, pred_label = argmax(logits),
     pred_score = prob[:, 1] (`test_video_segment_point.py:193-206`); optionally each window's vision
     embedding [T, 2048] is exported as vision_emb_{s}_{e}.npy (`convert2vision_emb.py:177-198`);
     BN: `--bn_mode running` (model.eval(), as convert2vision_emb.py:123 and the trainer's validation) or `batch`
     (test_video_segment_point.py:116-122: the running statistics are dropped and every batch of `batch_size`
     consecutive windows -- 16 there, :41 -- is normalised with its own statistics, so the batch partition is part
     of the result);
  5. runs of positive windows -> cut points (`eval_utils.py:3-18`, window step = stride) -> recall / precision
     at 0 / 3 / 5 s against the chapter starts (`eval_utils.py:21-92`) -> F.

usage: python long_video.py [--frames 3600] [--res 224] [--clip_frame_num 16] [--stride 1] [--batch_size 64]
                            [--bn_mode running|batch]
"""
import argparse
import json
import os
import random
import sys
import time

import numpy as np
import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
if _HERE not in sys.path:
    sys.path.insert(0, _HERE)

from data import clip_windows as cw  # noqa: E402
from eval_utils.eval_utils import calculate_pr, convert_clip_label2cut_point  # noqa: E402


def synthetic_long_video(n_frames=3600, H=224, W=224, chapter_every=300, seed=123, device="cuda"):
    """A synthetic 1 fps video: u8 frames [F, H, W, 3] on `device`, chapter timestamps about every
    `chapter_every` s ("m:ss title" strings, parsed by the reference's timestamp rules) and a subtitle about
    every 3 s. Frames are seeded noise (the model's weights are random too: the run measures the pipeline)."""
    g = torch.Generator(device="cpu").manual_seed(seed)
    frames = torch.randint(0, 256, (n_frames, H, W, 3), dtype=torch.uint8, generator=g).to(device)
    rng = random.Random(seed)
    t, timestamps = 0, []
    while t < n_frames:
        timestamps.append(f"{t // 3600}:{(t // 60) % 60:02d}:{t % 60:02d} chapter {len(timestamps)}")
        t += max(5, chapter_every // 3, int(rng.gauss(chapter_every, chapter_every / 5)))
    subtitles, s = [], 0.0
    while s < n_frames:
        subtitles.append({"start": round(s, 2),
                          "text": " ".join(f"w{rng.randint(0, 3000)}" for _ in range(rng.randint(2, 12)))})
        s += rng.uniform(1.0, 5.0)
    return frames, timestamps, subtitles


def window_inputs(n_frames, clip_frame_num, stride, subtitles, tokenizer, max_text_len):
    """Host-side integer / text work of every window: windows [n, 2], frame table [n, T] (0-based),
    token ids / masks [n, L]."""
    starts = np.arange(0, n_frames - clip_frame_num, stride, dtype=np.int64)
    win = np.stack([starts, starts + clip_frame_num], axis=1)
    idx = cw.frame_index_table(win, n_frames)
    ids = np.empty((len(win), max_text_len), dtype=np.int64)
    mask = np.empty_like(ids)
    for i, (s, e) in enumerate(win.tolist()):
        ids[i], mask[i] = cw.encode_text(tokenizer, cw.window_text(subtitles, s, e), max_text_len)
    return win, idx, ids, mask


@torch.no_grad()
def score_windows(model, frames_u8, idx, ids, mask, batch_size, export=None, streams=1, groups=1):
    """GPU part: per batch, frame gather + normalisation (ops.window_frames_u8) and the TwoStream forward.
    idx / ids / mask are device tensors. Returns (pred_score f32 [n], pred_label i64 [n]) on the device.
    export(b0, vision_emb [b, T, 2048]) is called per batch when given.
    streams > 1: consecutive batches go round-robin to that many HIP streams, so the small batches of the
    batch-statistics mode (16 windows: BN couples only the windows of one batch) run concurrently; every batch is
    still one forward over exactly its own windows, so the results are those of streams = 1.
    groups > 1: `groups` consecutive batches form one forward with per-batch BatchNorm statistics (TwoStream.bn_group
    = batch_size): BERT and the head run once over all of them; the results are those of groups = 1."""
    dt = model.compute_dtype()
    n = idx.shape[0]
    dev = frames_u8.device
    scores = torch.empty(n, dtype=torch.float32, device=dev)
    labels = torch.empty(n, dtype=torch.int64, device=dev)
    main = torch.cuda.current_stream(dev)
    pool = [main] if streams <= 1 or export is not None else [torch.cuda.Stream(device=dev) for _ in range(streams)]
    step = batch_size * max(1, groups)
    if groups > 1:
        if not hasattr(model, "bn_group"):
            raise ValueError("score_windows(groups > 1) needs a TwoStream model (per-group BatchNorm statistics)")
        saved_group, model.bn_group = model.bn_group, batch_size
    try:
        _score_batches(model, frames_u8, idx, ids, mask, n, step, dt, main, pool, scores, labels, export)
    finally:
        if groups > 1:
            model.bn_group = saved_group
    return scores, labels


def _score_batches(model, frames_u8, idx, ids, mask, n, step, dt, main, pool, scores, labels, export):
    from vcg_hip import ops
    for k, b0 in enumerate(range(0, n, step)):
        b1 = min(n, b0 + step)
        if k == 1 and len(pool) > 1:
            # batch 0 ran on the caller's stream: whatever the first forward prepares once (the bf16 weight shadow /
            # GEMM layouts / folded weights) is ordered before every stream's batches
            for s in pool:
                s.wait_stream(main)
        with torch.cuda.stream(main if k == 0 else pool[k % len(pool)]):
            fr = ops.window_frames_u8(frames_u8, idx[b0:b1].contiguous(), dt, cpad=ops.stem_cpad(dt))
            out = model.forward_staged(fr, ids[b0:b1], mask[b0:b1], return_emb=export is not None)
            logits, prob = out[0], out[1]
            scores[b0:b1] = prob[:, 1]
            labels[b0:b1] = logits.argmax(1)
        if export is not None:
            export(b0, out[2])
    for s in pool:
        if s is not main:
            main.wait_stream(s)


def boundary_metrics(labels, timestamps, n_frames, clip_frame_num, stride):
    """Cut points of the predicted window labels vs the ground-truth chapter starts (eval filter 4 <= cp <=
    F - 4, `flat_video2clip_for_quick_infer.py:52-57`): recall / precision / F at exact, 3 s and 5 s."""
    gt = cw.cut_points_from_timestamps(timestamps, n_frames, mode="eval")
    pred = convert_clip_label2cut_point(list(labels), clip_frame_num, stride / 2)
    if gt:
        r, r3, r5, p, p3, p5 = calculate_pr(gt, pred)
    else:  # no chapter start inside the scored range: recall is undefined (the reference would divide by 0)
        r = r3 = r5 = p = p3 = p5 = None

    def f(a, b):
        return 0.0 if (a is None or b is None or a + b == 0) else 2 * a * b / (a + b)
    return {"gt_cut_points": gt, "pred_cut_points": [int(c) for c in pred], "recall": r, "recall_3": r3,
            "recall_5": r5, "precision": p, "precision_3": p3, "precision_5": p5, "f": f(r, p), "f_3": f(r3, p3),
            "f_5": f(r5, p5)}


def main(argv=None):
    ap = argparse.ArgumentParser(description="long-video chapter-boundary inference (MI355X)")
    ap.add_argument("--gpu", default=0, type=int)
    ap.add_argument("--frames", default=3600, type=int, help="video length in frames (1 fps)")
    ap.add_argument("--res", default=224, type=int)
    ap.add_argument("--clip_frame_num", default=16, type=int)
    ap.add_argument("--stride", default=1, type=int)
    ap.add_argument("--max_text_len", default=128, type=int)
    ap.add_argument("--batch_size", default=None, type=int, help="default: 64 (running), 16 (batch, the test driver's)")
    ap.add_argument("--bn_mode", default="running", choices=["running", "batch"])
    ap.add_argument("--head_type", default="mlp", type=str)
    ap.add_argument("--precision", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--export_dir", default=None, help="write vision_emb_{s}_{e}.npy per window (convert2vision_emb)")
    ap.add_argument("--seed", default=123, type=int)
    args = ap.parse_args(argv)
    if args.batch_size is None:
        args.batch_size = 64 if args.bn_mode == "running" else 16

    from convert2vision_emb import emb_path
    from data.synthetic_dataset import HashTokenizer
    from vcg_hip import _lib
    from vcg_hip.build import build_two_stream

    dev = torch.device("cuda", args.gpu)
    torch.cuda.set_device(dev)
    _lib.call("vcg_init", args.gpu)
    model = build_two_stream(clip_frame_num=args.clip_frame_num, head_type=args.head_type, seed=args.seed,
                             device=dev, precision=args.precision).eval()
    if args.bn_mode == "batch":
        from test_video_segment_point import drop_bn_running_stats
        drop_bn_running_stats(model)
    frames, timestamps, subtitles = synthetic_long_video(args.frames, args.res, args.res, seed=args.seed, device=dev)
    win, idx, ids, mask = window_inputs(args.frames, args.clip_frame_num, args.stride, subtitles, HashTokenizer(),
                                        args.max_text_len)
    idx_d, ids_d, mask_d = (torch.from_numpy(a).to(dev) for a in (idx, ids, mask))
    export = None
    if args.export_dir:
        vid = "longvideo"
        os.makedirs(os.path.join(args.export_dir, vid), exist_ok=True)

        def export(b0, ve):
            ve = ve.float().cpu().numpy()
            for k in range(ve.shape[0]):
                s, e = win[b0 + k]
                np.save(emb_path(args.export_dir, vid, int(s), int(e)), ve[k])
    score_windows(model, frames, idx_d[:args.batch_size], ids_d[:args.batch_size], mask_d[:args.batch_size],
                  args.batch_size)  # warm-up
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    scores, labels = score_windows(model, frames, idx_d, ids_d, mask_d, args.batch_size, export)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    res = boundary_metrics(labels.cpu().tolist(), timestamps, args.frames, args.clip_frame_num, args.stride)
    res.update({"windows": int(len(win)), "seconds": dt, "windows_per_sec": len(win) / dt})
    print(json.dumps({k: v for k, v in res.items() if not k.endswith("cut_points")}))
    return res


if __name__ == "__main__":
    main()
