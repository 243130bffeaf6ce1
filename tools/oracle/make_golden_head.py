"""Goldens for ChapterHead head_type="attn" (reference model/fusion/two_stream.py:8-48, 63-67, 71-95),
produced by running the REFERENCE's own ChapterHead / TwoStream in this container (see make_golden.py;
only the .npz outputs are committed, the reference never travels).

tests/golden/head_attn.npz
  head_*  : a stand-alone reference ChapterHead(lang 96, vision 160, T=4, hidden 128, out 2, "attn"), eval
            (attn_drop inactive), weights from vcg_hip/synth.py by state-dict name (prefix "fusion_head."),
            inputs / loss weights from numpy's default_rng(7): logits, and the gradients of
            sum(logits * R) w.r.t. both inputs and every head parameter.
  c1attn_*: the full C1 TwoStream (T=4, 112^2, L=32, batch 2) with head_type="attn", running-stats eval with
            the calibrated BN statistics of bn_running_stats.npz: logits / prob.
usage: python tools/oracle/make_golden_head.py
"""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import make_golden as mg  # noqa: E402  (puts the reference on sys.path; loads vcg_hip/synth.py by path)

B, T, DL, DV, HID, O = 3, 4, 96, 160, 128, 2


def head_golden(out):
    head = mg.ref_two_stream.ChapterHead(DL, DV, T, HID, O, head_type="attn")
    mg.synth.init_params(head, mg.SEED, prefix="fusion_head.")
    head.eval()
    rng = np.random.default_rng(7)
    lang = torch.from_numpy(rng.standard_normal((B, DL)).astype(np.float32)).requires_grad_()
    vis = torch.from_numpy(rng.standard_normal((B, T, DV)).astype(np.float32)).requires_grad_()
    R = torch.from_numpy(rng.standard_normal((B, O)).astype(np.float32))
    logits = head(lang, vis)
    (logits * R).sum().backward()
    out.update({"head_lang": lang.detach().numpy(), "head_vis": vis.detach().numpy(), "head_R": R.numpy(),
                "head_logits": logits.detach().numpy(), "head_dlang": lang.grad.numpy(),
                "head_dvis": vis.grad.numpy()})
    for n, p in head.named_parameters():
        out[f"head_grad::{n}"] = p.grad.numpy()


def c1_golden(out):
    m = mg.build_reference(T=4, head_type="attn")
    stats = dict(np.load(os.path.join(mg.GOLD, "bn_running_stats.npz")))
    mg.synth.load_bn_stats(m, stats)
    frames, ids, mask, _ = mg.synth.clip_batch(2, 4, 112, 112, 32, seed=mg.SEED)
    m.eval()
    with torch.no_grad():
        lg, pr = m(frames, ids, mask)
    out.update({"c1attn_logits_running": lg.numpy(), "c1attn_prob_running": pr.numpy()})


def main():
    torch.set_num_threads(os.cpu_count() or 8)
    out = {}
    head_golden(out)
    c1_golden(out)
    np.savez_compressed(os.path.join(mg.GOLD, "head_attn.npz"), **out)
    print({k: v.shape for k, v in out.items()})


if __name__ == "__main__":
    main()
