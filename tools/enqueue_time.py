"""Host-side cost of one bench train step: wall time of step() until every launch is enqueued (no sync), and a
cProfile of one enqueue (top functions by own time). python tools/enqueue_time.py"""
import cProfile
import os
import pstats
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "video-chapter-generation_amd"))
sys.path.insert(0, REPO)


def main():
    from vcg_hip import _lib, synth
    from vcg_hip.build import build_two_stream
    from vcg_hip.functions import cross_entropy
    _lib.call("vcg_init", 0)
    dev = torch.device("cuda", 0)
    torch.manual_seed(123)
    model = build_two_stream(clip_frame_num=16, seed=123, device=dev, precision="bf16").train()

    class Cfg:
        weight_decay, learning_rate, betas = 0.01, 1e-5, (0.9, 0.95)
    opt = model.configure_optimizers(Cfg)
    frames, ids, mask, labels = synth.clip_batch(64, 16, 224, 224, 128, seed=123, device=dev)

    def step():
        opt.zero_grad()
        logits, _ = model(frames, ids, mask)
        cross_entropy(logits, labels).backward()
        opt.clip_and_step(1.0)

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    enq, tot = [], []
    for _ in range(10):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        step()
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        enq.append(1e3 * (t1 - t0))
        tot.append(1e3 * (t2 - t0))
    print("enqueue ms/step:", " ".join(f"{x:.1f}" for x in enq))
    print("total   ms/step:", " ".join(f"{x:.1f}" for x in tot))
    torch.cuda.synchronize()
    pr = cProfile.Profile()
    pr.enable()
    step()
    pr.disable()
    torch.cuda.synchronize()
    pstats.Stats(pr).sort_stats("tottime").print_stats(25)


if __name__ == "__main__":
    main()
