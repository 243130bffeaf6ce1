"""Diagnostic: TwoStream BERT gradients in bf16 with / without the BERT side stream, vs the fp32 native step."""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "video-chapter-generation_amd"))
sys.path.insert(0, REPO)
from vcg_hip import synth  # noqa: E402
from vcg_hip.build import build_two_stream  # noqa: E402
from vcg_hip.functions import cross_entropy  # noqa: E402

B, T, HW, L = 2, int(sys.argv[1]), int(sys.argv[2]), 128
frames, ids, mask, labels = synth.clip_batch(B, T, HW, HW, L, seed=11, device="cuda")


def run(prec, overlap, dlang_probe=False):
    m = build_two_stream(clip_frame_num=T, seed=123, device="cuda", precision=prec, dropout=0.0).train()
    m.overlap_streams = overlap
    lg, _, ve, le = m(frames, ids, mask, return_emb=True)
    le.retain_grad() if le.requires_grad else None
    loss = cross_entropy(lg, labels)
    loss.backward()
    torch.cuda.synchronize()
    g = {n: p.grad.detach().double().cpu() for n, p in m.named_parameters()}
    return loss.item(), lg.detach().double().cpu(), le.detach().double().cpu(), g


ref = run("fp32", True)
for prec, ov in (("fp32", False), ("bf16", True), ("bf16", False)):
    r = run(prec, ov)
    rel = lambda a, b: (a - b).norm().item() / max(b.norm().item(), 1e-300)  # noqa: E731
    e_b = np.array([rel(r[3][n], ref[3][n]) for n in ref[3] if n.startswith("lang_model") and ref[3][n].norm() > 1e-8])
    e_h = {n: rel(r[3][n], ref[3][n]) for n in ref[3] if n.startswith("fusion_head")}
    print(prec, "overlap" if ov else "single", "loss", r[0], "logits err", (r[1] - ref[1]).abs().max().item(),
          "lang_emb err", rel(r[2], ref[2]), "bert grad rel err median", np.median(e_b), "max", e_b.max(),
          "head", {k.split('.')[-2] + '.' + k.split('.')[-1]: round(v, 4) for k, v in e_h.items()}, flush=True)
