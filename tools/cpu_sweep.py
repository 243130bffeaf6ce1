"""CPU baseline measurements on the GPU box's host (the oracle, test infrastructure; bench.py's cpu_baseline):

  sweep: the oracle's fp32 eval forward (B = 4 windows) and train step (B = 2) at several torch thread counts, to
         show where the box's CPU share saturates (bench.py caps cpu_baseline at 16 threads);
  big:   the eval forward at B = 64 (config 2's batch) at the best thread count;
  c5:    config 5 on the CPU end to end at the reference's own stride (4 s: 896 windows of a 3600-frame 224^2 video,
         T = 16, L = 128), batch-statistics BN over batches of 16 consecutive windows (test_video_segment_point.py:41,
         116-122): frame gather + normalisation, tokenised text, the oracle forward, labels -> cut points -> F.

usage: python tools/cpu_sweep.py [sweep|train|big|c5|all ...] [--threads 1,4,8,16,32,64,128,0] [--out FILE]
(0 = every CPU this process may run on). Prints one JSON object per measurement."""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "video-chapter-generation_amd"))
sys.path.insert(0, REPO)


def _visible():
    try:
        return len(os.sched_getaffinity(0))
    except AttributeError:
        return os.cpu_count()


def _model(T):
    from vcg_hip.build import build_two_stream
    m = build_two_stream(clip_frame_num=T, dropout=0.1)
    sd = m.state_dict()
    names = [n for n, _ in m.named_parameters()]
    return sd, names


def time_fwd(sd, names, B, T, HW, L, threads, reps=2, bn="running"):
    import torch
    from oracle import model as om
    from vcg_hip import synth
    torch.set_num_threads(threads)
    frames, ids, mask, _ = synth.clip_batch(B, T, HW, HW, L, seed=7)
    p = dict(sd)
    ts = []
    for r in range(reps + 1):
        t0 = time.perf_counter()
        with torch.no_grad():
            om.two_stream(p, frames, ids, mask, bn_mode=bn)
        if r:
            ts.append(time.perf_counter() - t0)
    med = sorted(ts)[len(ts) // 2]
    return {"what": f"fwd {bn}-stat BN", "B": B, "threads": threads, "seconds": [round(t, 3) for t in ts],
            "windows_per_s": round(B / med, 4)}


def time_train(sd, names, B, T, HW, L, threads, reps=2):
    import torch
    from oracle import model as om
    from vcg_hip import synth
    torch.set_num_threads(threads)
    frames, ids, mask, labels = synth.clip_batch(B, T, HW, HW, L, seed=7)
    ts = []
    for r in range(reps + 1):
        params = {n: sd[n].detach().clone().requires_grad_(True) for n in names}
        buffers = {n: sd[n].detach().clone() for n in sd if n not in params}
        t0 = time.perf_counter()
        om.train_step(params, buffers, frames, ids, mask, labels, lr=1e-5)
        if r:
            ts.append(time.perf_counter() - t0)
    med = sorted(ts)[len(ts) // 2]
    return {"what": "train step", "B": B, "threads": threads, "seconds": [round(t, 3) for t in ts],
            "windows_per_s": round(B / med, 4)}


def c5(threads, F=3600, T=16, HW=224, L=128, stride=4, BS=16):
    import numpy as np
    import torch
    import long_video as lv
    from data.synthetic_dataset import HashTokenizer, normalize_frames
    from oracle import model as om
    from vcg_hip.build import build_two_stream
    torch.set_num_threads(threads)
    m = build_two_stream(clip_frame_num=T, seed=123, dropout=0.0)
    p = {k: v for k, v in m.state_dict().items() if "running" not in k and "num_batches" not in k}
    t_all = time.perf_counter()
    frames, timestamps, subtitles = lv.synthetic_long_video(F, HW, HW, seed=123, device="cpu")
    fr = frames.numpy()
    win, idx, ids, mask = lv.window_inputs(F, T, stride, subtitles, HashTokenizer(), L)
    labels = []
    t_fwd = 0.0
    for b0 in range(0, len(win), BS):
        sel = slice(b0, min(len(win), b0 + BS))
        img = normalize_frames(fr[idx[sel]])
        t0 = time.perf_counter()
        with torch.no_grad():
            logits, _, _, _ = om.two_stream(p, img, torch.from_numpy(ids[sel]), torch.from_numpy(mask[sel]),
                                            bn_mode="batch")
        t_fwd += time.perf_counter() - t0
        labels += logits.argmax(1).tolist()
        if (b0 // BS) % 8 == 0:
            print(f"c5: {b0 + BS}/{len(win)} windows, {time.perf_counter() - t_all:.1f} s", flush=True)
    met = lv.boundary_metrics(labels, timestamps, F, T, stride)
    sec = time.perf_counter() - t_all
    return {"what": "config 5 on the CPU (oracle): 1 h synthetic video, stride 4 s, batch-stat BN in batches of 16",
            "windows": len(win), "threads": threads, "seconds_end_to_end": round(sec, 2),
            "seconds_forward": round(t_fwd, 2), "windows_per_s": round(len(win) / sec, 4),
            "boundary": {k: met[k] for k in ("recall", "precision", "f", "f_3", "f_5")}}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("what", nargs="*", default=["all"], help="sweep / train / big / c5 / all")
    ap.add_argument("--threads", default="1,4,8,16,32,64,128,0")
    ap.add_argument("--c5-threads", type=int, default=0, help="0: the sweep's best forward thread count")
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    vis = _visible()
    th = sorted({(vis if int(t) == 0 else int(t)) for t in args.threads.split(",") if int(t) <= vis})
    out = open(args.out, "a") if args.out else None

    def emit(d):
        d.update(cpu_visible=vis, cpu_count=os.cpu_count())
        line = json.dumps(d)
        print(line, flush=True)
        if out:
            out.write(line + "\n")
            out.flush()
    T, HW, L = 16, 224, 128
    sd, names = _model(T)
    best = 16
    what = set(args.what)
    if what & {"sweep", "all"}:
        res = []
        for t in th:
            r = time_fwd(sd, names, 4, T, HW, L, t)
            emit(r)
            res.append(r)
        best = max(res, key=lambda r: r["windows_per_s"])["threads"]
    if what & {"sweep", "train", "all"}:
        for t in sorted({16, best} | set(th if "train" in what else ())):
            emit(time_train(sd, names, 2, T, HW, L, t))
    if what & {"big", "all"}:
        emit(time_fwd(sd, names, 64, T, HW, L, args.c5_threads or best, reps=1))
    if what & {"c5", "all"}:
        emit(c5(args.c5_threads or best))


if __name__ == "__main__":
    main()
