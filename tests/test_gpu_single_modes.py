"""Text-only and image-only modes (`--data_mode text|image`) on libvcg_hip against the CPU
oracle: BertHugface.forward (reference model/lang/bert_hugface.py:98-132: pooler_output -> head -> softmax),
Resnet50TSM.forward (model/vision/resnet50_tsm.py:68-77: frames -> TSM-ResNet-50 -> [B, T*2048] -> head ->
softmax) and the plain Resnet50 (model/vision/resnet50.py:65-73).

Tolerances: fp32 parity mode -- logits / prob within 1e-3; every parameter gradient as close to the exact
(fp64) oracle gradient as the oracle's own fp32 (reference-arithmetic) gradient is: relative Frobenius error
<= max(3 x the fp32 oracle's, 2e-3). (The vision trunk at B=2, T=4, 112² with BatchNorm batch statistics over
8 frames amplifies fp32 rounding to ~1e-2 on many tensors -- the reference's own arithmetic does the same.)
Analytically-zero gradients (attention key biases: softmax is shift-invariant) are only checked to be tiny.
bf16 -- logits within 5e-2.
"""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _oracle_params(model_cpu, dtype=torch.float32):
    sd = model_cpu.state_dict()
    names = [n for n, _ in model_cpu.named_parameters()]
    params = {n: sd[n].detach().to(dtype).clone().requires_grad_() for n in names}
    p = {n: (sd[n].detach().to(dtype).clone() if sd[n].is_floating_point() else sd[n]) for n in sd if n not in params}
    p.update(params)
    return p, params


def _check_grads(model, ref32, ref64):
    """ours vs exact within max(5 x |oracle fp32 - exact|, 2e-3) and 5e-2 (relative Frobenius) per tensor. In the
    batch-statistics regime the rounding error of any fp32 implementation is amplified ~1e5 and depends on its
    summation orders: the SAME torch oracle changes its error vs exact by 4x (median) between 1 and 8 CPU threads,
    and a 1e-7 input perturbation moves it by up to 2.4x (measured at this shape); ours / oracle-fp32 reaches ~3.4
    on layer1-2 BatchNorm parameters of the TSM trunk."""
    gmax = max(v.grad.double().norm().item() for v in ref64.values() if v.grad is not None)
    bad, ratios = [], []
    for n, prm in model.named_parameters():
        r64 = ref64[n].grad
        if r64 is None:
            continue
        a, b = prm.grad.detach().double().cpu().reshape(-1), r64.double().reshape(-1)
        nb = b.norm().item()
        if nb <= 1e-6 * gmax:  # analytically zero (e.g. attention key bias): ours must be tiny too
            assert a.norm().item() <= 1e-5 * gmax, n
            continue
        e = (a - b).norm().item() / nb
        e_ref = (ref32[n].grad.double().reshape(-1) - b).norm().item() / nb
        ratios.append(e / max(e_ref, 2e-3 / 5))
        if e > max(5 * e_ref, 2e-3) or e > 5e-2:
            bad.append((n, e, e_ref))
    print(f"grad error ratio ours / oracle-fp32: median {np.median(ratios):.2f} max {max(ratios):.2f}")
    assert not bad, f"{len(bad)} of {len(ratios)} gradients off (ours, oracle fp32): {bad[:5]}"


@pytest.mark.parametrize("precision", ["fp32", "bf16"])
def test_text_only_mode(precision):
    from oracle import model as om
    from vcg_hip import synth
    from vcg_hip.build import build_model
    from vcg_hip.functions import cross_entropy
    torch.set_num_threads(min(16, os.cpu_count() or 8))
    B, L = 4, 32
    _, ids, mask, labels = synth.clip_batch(B, 1, 8, 8, L, seed=21, device=DEV)
    m = build_model("text", seed=123, device=DEV, precision=precision, dropout=0.0).train()
    cpu = build_model("text", seed=123, precision=precision, dropout=0.0)
    refs = {}
    for dt in (torch.float32, torch.float64):
        p, params = _oracle_params(cpu, dt)
        pooled, _ = om.bert(p, ids.cpu(), mask.cpu(), prefix="base_model.")
        lg, pr = om.linear_head(p, pooled)
        ce = torch.nn.functional.cross_entropy(lg, labels.cpu())
        ce.backward()
        refs[dt] = (lg.detach().float(), pr.detach().float(), ce.item(), params)
    ref_logits, ref_prob, ce_ref, _ = refs[torch.float64]
    logits, prob = m(ids, mask)
    loss = cross_entropy(logits, labels)
    loss.backward()
    torch.cuda.synchronize()
    tol = 1e-3 if precision == "fp32" else 5e-2
    assert (logits.detach().cpu() - ref_logits).abs().max().item() <= tol
    assert (prob.detach().cpu() - ref_prob).abs().max().item() <= tol
    assert abs(loss.item() - ce_ref) <= tol
    if precision == "fp32":
        _check_grads(m, refs[torch.float32][3], refs[torch.float64][3])


@pytest.mark.parametrize("model_type", ["r50tsm", "r50"])
def test_image_only_mode(model_type):
    from oracle import model as om
    from vcg_hip import synth
    from vcg_hip.build import build_model
    from vcg_hip.functions import cross_entropy
    torch.set_num_threads(min(16, os.cpu_count() or 8))
    B, T, HW = 2, 4, 112
    frames, _, _, labels = synth.clip_batch(B, T, HW, HW, 8, seed=22, device=DEV)
    m = build_model("image", clip_frame_num=T, model_type=model_type, seed=123, device=DEV, precision="fp32").train()
    cpu = build_model("image", clip_frame_num=T, model_type=model_type, seed=123, precision="fp32")
    refs = {}
    for dt in (torch.float32, torch.float64):
        p, params = _oracle_params(cpu, dt)
        emb = om.resnet50_tsm(p, frames.cpu().to(dt).reshape(B * T, 3, HW, HW), T, "train", prefix="base_model.",
                              tsm=model_type == "r50tsm")
        lg, pr = om.linear_head(p, emb.reshape(B, -1))
        ce = torch.nn.functional.cross_entropy(lg, labels.cpu())
        ce.backward()
        refs[dt] = (lg.detach().float(), pr.detach().float(), ce.item(), params, p)
    ref_logits, ref_prob, ref_loss, _, p = refs[torch.float64]
    logits, prob = m(frames)
    loss = cross_entropy(logits, labels)
    loss.backward()
    torch.cuda.synchronize()
    assert (logits.detach().cpu() - ref_logits).abs().max().item() <= 1e-3
    assert (prob.detach().cpu() - ref_prob).abs().max().item() <= 1e-3
    assert abs(loss.item() - ref_loss) <= 1e-4
    _check_grads(m, refs[torch.float32][3], refs[torch.float64][3])
    # running statistics were updated like the oracle's F.batch_norm(training=True)
    bufs = dict(m.named_buffers())
    for n, b in p.items():
        if n.endswith("running_mean") or n.endswith("running_var"):
            assert (bufs[n].cpu().double() - b).abs().max().item() <= 1e-4 * (1 + b.abs().max().item()), n


def test_image_only_mode_bf16_forward():
    from oracle import model as om
    from vcg_hip import synth
    from vcg_hip.build import build_model
    B, T, HW = 2, 4, 112
    frames, _, _, _ = synth.clip_batch(B, T, HW, HW, 8, seed=23, device=DEV)
    m = build_model("image", clip_frame_num=T, seed=123, device=DEV, precision="bf16").eval()
    for mod in m.modules():  # batch-statistics eval (test_video_segment_point.py:116-122)
        if isinstance(mod, torch.nn.BatchNorm2d):
            mod.track_running_stats, mod.running_mean, mod.running_var = False, None, None
    cpu = build_model("image", clip_frame_num=T, seed=123, precision="bf16")
    p, _ = _oracle_params(cpu)
    with torch.no_grad():
        emb = om.resnet50_tsm(p, frames.cpu().reshape(B * T, 3, HW, HW), T, "batch", prefix="base_model.")
        ref_logits, _ = om.linear_head(p, emb.reshape(B, -1))
        logits, _ = m(frames)
    assert (logits.cpu() - ref_logits).abs().max().item() <= 5e-2
