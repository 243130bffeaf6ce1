"""tests/golden/c1_train_fp64.npz: exact-arithmetic (fp64) C1 train-step gradients from the oracle.

The reference's fp32 train-step gradients (c1_train.npz) carry fp32 noise of up to a few percent
elementwise on vision BatchNorm-adjacent tensors (8-frame batch statistics, ReLU / max-pool
boundaries). The GPU parity test therefore measures both the reference fp32 and libvcg_hip fp32
against these fp64 gradients and requires libvcg_hip to be as close to exact as the reference is.
The oracle itself is pinned to the reference by tests/test_cpu_oracle.py.
Usage: python tools/oracle/make_fp64_grads.py
"""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "video-chapter-generation_amd"))
sys.path.insert(0, REPO)

from oracle import model as om  # noqa: E402
from vcg_hip import synth  # noqa: E402
from vcg_hip.build import build_two_stream  # noqa: E402


def main():
    gold = os.path.join(REPO, "tests", "golden")
    g = np.load(os.path.join(gold, "c1_train.npz"))
    torch.set_num_threads(os.cpu_count() or 8)
    m = build_two_stream(clip_frame_num=4, seed=123, bn_stats=dict(np.load(os.path.join(gold, "bn_running_stats.npz"))),
                         dropout=0.0)
    sd = m.state_dict()
    names = [n for n, _ in m.named_parameters()]
    params = {n: sd[n].detach().double().clone().requires_grad_() for n in names}
    buffers = {n: (sd[n].detach().double().clone() if sd[n].is_floating_point() else sd[n]) for n in sd
               if n not in params}
    frames, ids, mask, labels = synth.clip_batch(2, 4, 112, 112, 32, seed=123)
    p = dict(buffers)
    p.update(params)
    logits, _, _, _ = om.two_stream(p, frames.double(), ids, mask, bn_mode="train")
    loss = torch.nn.functional.cross_entropy(logits, labels)
    loss.backward()
    out = {"loss": np.array([loss.item()]), "norm_names": np.array(names),
           "norms": np.array([params[n].grad.norm().item() for n in names])}
    for key in [k for k in g.files if k.startswith("train_grad::")]:
        n = key.split("::", 1)[1]
        out[f"grad::{n}"] = params[n].grad.reshape(-1)[g[f"train_idx::{n}"]].numpy()
    np.savez_compressed(os.path.join(gold, "c1_train_fp64.npz"), **out)
    print("wrote c1_train_fp64.npz, loss", loss.item())


if __name__ == "__main__":
    main()
