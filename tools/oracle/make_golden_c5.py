"""Generate tests/golden/c5_stride4_batch16.npz: BASELINE config 5 end to end on the CPU ORACLE (test infrastructure).

The reference's F1 pipeline (test_video_segment_point.py:244-377 -> eval_utils.py:3-92) at the reference's own window
stride (2 * max_offset = 4 s, flat_video2clip_for_quick_infer.py:66) over the config-5 synthetic video
(long_video.synthetic_long_video: 3600 frames of 224^2, seed 123), T = 16, L = 128, batch-statistics BN in batches of
16 consecutive windows (test_video_segment_point.py:41,116-122): 896 windows, 56 batches, fp32.

Model: build_two_stream(seed=123) random-init weights (vcg_hip/synth.py: numpy here, the bit-identical HIP generator on
the GPU box), running statistics dropped. The random-init 2-way head puts every window on one side of 0.5, so logit 1's
bias is shifted by the median logit margin of the first batch (computed here by the oracle, stored in the fixture and
applied unchanged by the GPU test).

Stored: per-window prob[:, 1] (f64), predicted labels, the windows, the bias shift and the boundary metrics
(long_video.boundary_metrics = eval_utils' cut points / P-R at 0 / 3 / 5 s) of the oracle's labels.
Runs ~13 min on 8 CPU threads:  python tools/oracle/make_golden_c5.py [--threads 8]
"""
import argparse
import os
import sys
import time

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "video-chapter-generation_amd"))
sys.path.insert(0, REPO)

F, T, HW, L, STRIDE, BS = 3600, 16, 224, 128, 4, 16
OUT = os.path.join(REPO, "tests", "golden", "c5_stride4_batch16.npz")
METRIC_KEYS = ("recall", "recall_3", "recall_5", "precision", "precision_3", "precision_5", "f", "f_3", "f_5")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--limit", type=int, default=0, help="score only this many batches (smoke runs)")
    args = ap.parse_args()
    torch.set_num_threads(args.threads)
    import long_video as lv
    from data.synthetic_dataset import HashTokenizer, normalize_frames
    from oracle import model as om
    from test_video_segment_point import drop_bn_running_stats
    from vcg_hip.build import build_two_stream

    frames, timestamps, subtitles = lv.synthetic_long_video(F, HW, HW, seed=123, device="cpu")
    win, idx, ids, mask = lv.window_inputs(F, T, STRIDE, subtitles, HashTokenizer(), L)
    assert len(win) == 896, len(win)
    model = build_two_stream(clip_frame_num=T, seed=123, device="cpu", precision="fp32", dropout=0.0).eval()
    assert drop_bn_running_stats(model) == 53
    fr_np = frames.numpy()

    def batch(b0, p):
        sel = np.arange(b0, min(len(win), b0 + BS))
        img = normalize_frames(fr_np[idx[sel]])
        with torch.no_grad():
            lg, pr, _, _ = om.two_stream(p, img, torch.from_numpy(ids[sel]), torch.from_numpy(mask[sel]),
                                         bn_mode="batch")
        return lg, pr

    p = {k: v.detach().clone() for k, v in model.state_dict().items()}
    lg0, _ = batch(0, p)
    shift = float((lg0[:, 0] - lg0[:, 1]).median().item())
    with torch.no_grad():
        model.fusion_head.head.bias.data[1] += shift
    p = {k: v.detach().clone() for k, v in model.state_dict().items()}
    starts = list(range(0, len(win), BS))
    if args.limit:
        starts = starts[:args.limit]
    prob = np.full(len(win), np.nan)
    labels = np.full(len(win), -1, dtype=np.int64)
    t0 = time.time()
    for k, b0 in enumerate(starts):
        lg, pr = batch(b0, p)
        prob[b0:b0 + len(pr)] = pr[:, 1].double().numpy()
        labels[b0:b0 + len(pr)] = lg.argmax(1).numpy()
        print(f"batch {k + 1}/{len(starts)}  {time.time() - t0:.0f} s", flush=True)
    out = {"prob1": prob, "labels": labels, "win": win, "shift": np.float64(shift),
           "config": np.array([F, T, HW, L, STRIDE, BS], dtype=np.int64)}
    if not args.limit:
        m = lv.boundary_metrics(labels.tolist(), timestamps, F, T, STRIDE)
        for k in METRIC_KEYS:
            out["metric_" + k] = np.float64(np.nan if m[k] is None else m[k])
        out["gt_cut_points"] = np.array(m["gt_cut_points"], dtype=np.int64)
        out["pred_cut_points"] = np.array(m["pred_cut_points"], dtype=np.int64)
        print({k: m[k] for k in METRIC_KEYS}, "positive share", labels.mean())
        np.savez_compressed(OUT, **out)
        print("wrote", OUT)


if __name__ == "__main__":
    main()
