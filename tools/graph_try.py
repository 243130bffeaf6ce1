"""Feasibility of capturing the bench train step in one HIP graph (torch.cuda.CUDAGraph): eager vs replay
ms/step and CPU time per step. python tools/graph_try.py"""
import os
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
    out = {}

    def step():
        opt.zero_grad()
        logits, _ = model(frames, ids, mask)
        loss = cross_entropy(logits, labels)
        loss.backward()
        opt.clip_and_step(1.0)
        out["loss"] = loss

    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            step()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()

    def timed(fn, n):
        torch.cuda.synchronize()
        t0, c0 = time.perf_counter(), time.process_time()
        for _ in range(n):
            fn()
        torch.cuda.synchronize()
        return 1e3 * (time.perf_counter() - t0) / n, 1e3 * (time.process_time() - c0) / n

    print("eager: %.2f ms/step, cpu %.2f ms/step" % timed(step, 10), flush=True)
    g = torch.cuda.CUDAGraph()
    t0 = time.perf_counter()
    with torch.cuda.graph(g):
        step()
    torch.cuda.synchronize()
    print("captured in %.1f s" % (time.perf_counter() - t0), flush=True)
    print("replay: %.2f ms/step, cpu %.2f ms/step" % timed(g.replay, 20), flush=True)
    g.replay()
    torch.cuda.synchronize()
    print("loss after replays", float(out["loss"]), flush=True)
    print("eager again: %.2f ms/step, cpu %.2f ms/step" % timed(step, 5), flush=True)


if __name__ == "__main__":
    main()
