"""Diagnostic: BERT (text-only mode) gradients, native bf16 / fp32 vs the exact oracle and torch autocast."""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "video-chapter-generation_amd"))
sys.path.insert(0, REPO)
from oracle import model as om  # noqa: E402
from vcg_hip import synth  # noqa: E402
from vcg_hip.build import build_model  # noqa: E402
from vcg_hip.functions import cross_entropy  # noqa: E402

torch.set_num_threads(16)
B, L = int(sys.argv[1]) if len(sys.argv) > 1 else 2, 128
_, ids, mask, labels = synth.clip_batch(B, 1, 8, 8, L, seed=11)
cpu = build_model("text", seed=123, precision="fp32", dropout=0.0)
sd = cpu.state_dict()
names = [n for n, _ in cpu.named_parameters()]


def oracle(dt, ac=False):
    params = {n: sd[n].detach().to(dt).clone().requires_grad_() for n in names}
    p = {n: (sd[n].detach().to(dt).clone() if sd[n].is_floating_point() else sd[n]) for n in sd if n not in params}
    p.update(params)
    with torch.autocast("cpu", dtype=torch.bfloat16, enabled=ac):
        pooled, _ = om.bert(p, ids, mask, prefix="base_model.")
        lg, _ = om.linear_head(p, pooled.float() if ac else pooled)
        loss = torch.nn.functional.cross_entropy(lg.float(), labels)
    loss.backward()
    return {n: params[n].grad.double() for n in names}, pooled.detach().double()


g64, p64 = oracle(torch.float64)
gac, pac = oracle(torch.float32, True)
res = {}
for prec in ("fp32", "bf16"):
    m = build_model("text", seed=123, device="cuda", precision=prec, dropout=0.0).train()
    lg, _ = m(ids.cuda(), mask.cuda())
    cross_entropy(lg, labels.cuda()).backward()
    torch.cuda.synchronize()
    res[prec] = {n: p.grad.detach().double().cpu() for n, p in m.named_parameters()}
    pooled = m.base_model(input_ids=ids.cuda(), attention_mask=mask.cuda()).pooler_output.double().cpu()
    print(prec, "pooled rel err", ((pooled - p64).norm() / p64.norm()).item())
print("autocast pooled rel err", ((pac - p64).norm() / p64.norm()).item())


def rel(a, b):
    return (a - b).norm().item() / max(b.norm().item(), 1e-300)


gmax = max(v.norm().item() for v in g64.values())
rows = []
for n in names:
    if g64[n].norm().item() <= 1e-6 * gmax:
        continue
    rows.append((n, rel(res["fp32"][n], g64[n]), rel(res["bf16"][n], g64[n]), rel(gac[n], g64[n]),
                 rel(res["bf16"][n], gac[n])))
rows.sort(key=lambda r: -r[2])
print(f"{'tensor':60s} fp32  bf16  autocast  bf16-vs-autocast")
for r in rows[:30]:
    print(f"{r[0]:60s} {r[1]:.2e} {r[2]:.2e} {r[3]:.2e} {r[4]:.2e}")
a = np.array([r[2] for r in rows])
b = np.array([r[3] for r in rows])
print("median bf16", np.median(a), "autocast", np.median(b))
