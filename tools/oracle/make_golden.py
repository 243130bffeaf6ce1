"""Generate tests/golden/* by running the REFERENCE's own modules in this container.

Runs only here (the reference never travels to the GPU box; only the .npz/.json outputs are
committed). Imports by path from /root/reference/video_chapter_generation:
  model.fusion.two_stream (TwoStream, ChapterHead), ops.temporal_shift (TemporalShift),
  eval_utils.eval_utils (convert_clip_label2cut_point, calculate_pr)
and uses transformers' BertModel (eager attention) as lang_model. torchvision is absent, so the
ResNet-50 trunk is tools/oracle/tv_resnet.py with reference TemporalShift wrappers inserted exactly
as make_temporal_shift(place='blockres') does (ops/temporal_shift.py:128-144).

Weights and inputs come from the counter-based generator in vcg_hip/synth.py (bit-identical on
the GPU box), so only outputs need committing. Usage:  python tools/oracle/make_golden.py [--skip-c2]
"""
import argparse
import copy
import json
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference/video_chapter_generation"
GOLD = os.path.join(REPO, "tests", "golden")
sys.path.insert(0, REF)  # reference packages (model, ops, eval_utils: namespace packages) first
sys.path.insert(1, HERE)


def _load_by_path(name, path):
    # our own package dir is NOT put on sys.path: its regular packages (model/, ops/, eval_utils/)
    # would shadow the reference's namespace packages of the same names
    import importlib.util
    spec = importlib.util.spec_from_file_location(name, path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


from model.fusion import two_stream as ref_two_stream  # noqa: E402
from ops.temporal_shift import TemporalShift  # noqa: E402
from eval_utils.eval_utils import calculate_pr, convert_clip_label2cut_point  # noqa: E402
import tv_resnet  # noqa: E402

synth = _load_by_path("vcg_synth", os.path.join(REPO, "video-chapter-generation_amd", "vcg_hip", "synth.py"))

SEED = 123
TRACKED = [
    "fusion_head.head.weight", "fusion_head.head.bias", "fusion_head.vision_proj_head.weight",
    "fusion_head.lang_proj_head.weight", "lang_model.pooler.dense.weight", "lang_model.pooler.dense.bias",
    "lang_model.encoder.layer.11.output.dense.weight", "lang_model.encoder.layer.11.output.LayerNorm.weight",
    "lang_model.encoder.layer.0.attention.self.query.weight", "lang_model.encoder.layer.0.attention.self.value.bias",
    "lang_model.embeddings.word_embeddings.weight", "lang_model.embeddings.position_embeddings.weight",
    "lang_model.embeddings.token_type_embeddings.weight", "lang_model.embeddings.LayerNorm.weight",
    "vision_model.layer4.2.conv3.weight", "vision_model.layer4.2.bn3.weight", "vision_model.layer3.0.conv2.weight",
    "vision_model.layer1.0.conv1.net.weight", "vision_model.layer1.0.downsample.0.weight",
    "vision_model.layer1.0.downsample.1.bias", "vision_model.conv1.weight", "vision_model.bn1.weight",
    "vision_model.bn1.bias",
]


def sample_idx(n, k=256):
    return np.unique(np.linspace(0, n - 1, num=min(k, n)).astype(np.int64))


def build_reference(T, dropout=0.0, head_type="mlp"):
    from transformers import BertConfig, BertModel
    cfg = BertConfig(output_attentions=True, hidden_dropout_prob=dropout, attention_probs_dropout_prob=dropout)
    cfg._attn_implementation = "eager"
    lang = BertModel(cfg, add_pooling_layer=True)
    vis = tv_resnet.ResNet()
    for layer in (vis.layer1, vis.layer2, vis.layer3, vis.layer4):  # blockres, n_round = 1
        for b in layer:
            b.conv1 = TemporalShift(b.conv1, n_segment=T, n_div=8)
    vis.fc = torch.nn.Identity()
    m = ref_two_stream.TwoStream(lang, vis, 768, 2048, T, 128)
    m.build_chapter_head(output_size=2, head_type=head_type)
    synth.init_params(m, SEED)
    return m


def calibrate_bn(m, seed_name="calib"):
    """Running stats := batch statistics of a calibration batch (a 'trained-like' BN state)."""
    frames, _, _, _ = synth.clip_batch(2, m.segment_size, 112, 112, 32, seed=seed_name)
    bns = [x for x in m.modules() if isinstance(x, torch.nn.BatchNorm2d)]
    for b in bns:
        b.momentum = 1.0
    m.vision_model.train()
    with torch.no_grad():
        m.vision_model(frames.view(-1, 3, 112, 112))
    for b in bns:
        b.momentum = 0.1
        b.num_batches_tracked.zero_()
    return {n: b.detach().numpy().copy() for n, b in m.named_buffers()
            if n.endswith("running_mean") or n.endswith("running_var")}


def batch_mode(m):
    """test_video_segment_point.py:116-122: BN uses batch statistics in eval."""
    m = copy.deepcopy(m)
    for mod in m.modules():
        if isinstance(mod, torch.nn.BatchNorm2d):
            mod.track_running_stats = False
            mod.running_mean = None
            mod.running_var = None
    return m


def fwd_golden(m, B, T, HW, L, tag, out):
    frames, ids, mask, labels = synth.clip_batch(B, T, HW, HW, L, seed=SEED)
    m.eval()
    with torch.no_grad():
        lg, pr, ve, le = m(frames, ids, mask, return_emb=True)
        mb = batch_mode(m)
        lgb, prb, veb, leb = mb(frames, ids, mask, return_emb=True)
    out.update({f"{tag}_logits_running": lg.numpy(), f"{tag}_prob_running": pr.numpy(),
                f"{tag}_logits_batch": lgb.numpy(), f"{tag}_prob_batch": prb.numpy(),
                f"{tag}_lang_emb": le.numpy(), f"{tag}_labels": labels.numpy(),
                f"{tag}_frames_checksum": np.array([frames.double().sum().item(), frames.double().abs().sum().item()]),
                f"{tag}_ids": ids.numpy(), f"{tag}_mask": mask.numpy()})
    if B * T <= 16:
        out[f"{tag}_vision_emb_running"] = ve.numpy()
        out[f"{tag}_vision_emb_batch"] = veb.numpy()
    else:
        out[f"{tag}_vision_emb_running_rows"] = ve.reshape(B * T, -1)[::37].numpy()
        out[f"{tag}_vision_emb_batch_rows"] = veb.reshape(B * T, -1)[::37].numpy()


def train_golden(m, out, lr=1e-4):
    B, T, HW, L = 2, 4, 112, 32
    frames, ids, mask, labels = synth.clip_batch(B, T, HW, HW, L, seed=SEED)
    m.train()
    before = {n: p.detach().clone() for n, p in m.named_parameters()}

    class Cfg:
        weight_decay = 0.01
        learning_rate = lr
        betas = (0.9, 0.95)
    opt = m.configure_optimizers(Cfg)
    logits, prob = m(frames, ids, mask)
    loss = torch.nn.functional.cross_entropy(logits, labels)
    loss.backward()
    grads = {n: p.grad.detach().clone() for n, p in m.named_parameters()}
    total = torch.nn.utils.clip_grad_norm_(m.parameters(), 1.0)
    opt.step()
    out["train_loss"] = np.array([loss.item()])
    out["train_logits"] = logits.detach().numpy()
    out["train_total_norm"] = np.array([total.item()])
    out["train_lr"] = np.array([lr])
    names = [n for n, _ in m.named_parameters()]
    out["train_grad_norm_names"] = np.array(names)
    out["train_grad_norms"] = np.array([grads[n].double().norm().item() for n in names])
    for n in TRACKED:
        g = grads[n].reshape(-1)
        idx = sample_idx(g.numel())
        p = dict(m.named_parameters())[n]
        out[f"train_idx::{n}"] = idx
        out[f"train_grad::{n}"] = g[idx].numpy()
        out[f"train_delta::{n}"] = (p.detach().reshape(-1)[idx] - before[n].reshape(-1)[idx]).numpy()
        out[f"train_exp_avg::{n}"] = opt.state[p]["exp_avg"].reshape(-1)[idx].numpy()
    bufs = dict(m.named_buffers())
    for n in ["vision_model.bn1", "vision_model.layer4.2.bn3", "vision_model.layer2.0.downsample.1"]:
        out[f"train_rm::{n}"] = bufs[n + ".running_mean"].numpy()
        out[f"train_rv::{n}"] = bufs[n + ".running_var"].numpy()


def tsm_golden(out):
    x = torch.from_numpy(synth.fill_np(8 * 64 * 7 * 7, synth.KIND_NORMAL, synth.key_of(SEED, "tsm_x"), 0, 1))
    x = x.view(8, 64, 7, 7).requires_grad_()
    y = TemporalShift.shift(x, 4, fold_div=8)
    g = torch.from_numpy(synth.fill_np(y.numel(), synth.KIND_NORMAL, synth.key_of(SEED, "tsm_g"), 0, 1)).view_as(y)
    (gx,) = torch.autograd.grad(y, x, g)
    out["tsm_x"] = x.detach().numpy()
    out["tsm_y"] = y.detach().numpy()
    out["tsm_g"] = g.numpy()
    out["tsm_gx"] = gx.numpy()


def eval_golden():
    rng = np.random.RandomState(SEED)
    cases = [{"labels": [1, 0, 0, 0, 1, 1, 0, 0, 1, 1, 1, 1, 1, 0, 1, 0, 0, 0, 0, 1, 1], "T": 16, "off": 2}]
    for _ in range(40):
        n = int(rng.randint(0, 60))
        cases.append({"labels": rng.randint(0, 2, size=n).tolist(), "T": int(rng.choice([8, 16, 32])),
                      "off": int(rng.choice([1, 2, 4]))})
    for c in cases:
        c["cut_points"] = convert_clip_label2cut_point(c["labels"], c["T"], c["off"])
    pr_cases = [{"gt": [10, 50, 90], "pred": [11, 48, 200]}, {"gt": [5], "pred": []}]
    for _ in range(40):
        gt = sorted(rng.randint(0, 600, size=int(rng.randint(1, 8))).tolist())
        pred = sorted(rng.randint(0, 600, size=int(rng.randint(0, 8))).tolist())
        pr_cases.append({"gt": gt, "pred": pred})
    for c in pr_cases:
        c["pr"] = list(calculate_pr(c["gt"], c["pred"]))
    return {"convert_clip_label2cut_point": cases, "calculate_pr": pr_cases}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--skip-c2", action="store_true")
    args = ap.parse_args()
    torch.set_num_threads(os.cpu_count() or 8)
    os.makedirs(GOLD, exist_ok=True)

    out = {}
    tsm_golden(out)
    np.savez_compressed(os.path.join(GOLD, "tsm_shift.npz"), **out)
    with open(os.path.join(GOLD, "eval_utils.json"), "w") as f:
        json.dump(eval_golden(), f)

    m = build_reference(T=4)
    stats = calibrate_bn(m)
    np.savez_compressed(os.path.join(GOLD, "bn_running_stats.npz"), **stats)
    out = {}
    fwd_golden(m, 2, 4, 112, 32, "c1", out)
    np.savez_compressed(os.path.join(GOLD, "c1_fwd.npz"), **out)
    out = {}
    train_golden(m, out)
    np.savez_compressed(os.path.join(GOLD, "c1_train.npz"), **out)
    print("c1 done")

    if not args.skip_c2:
        m = build_reference(T=16)
        synth.load_bn_stats(m, stats)
        out = {}
        fwd_golden(m, 64, 16, 224, 128, "c2", out)
        np.savez_compressed(os.path.join(GOLD, "c2_fwd.npz"), **out)
        print("c2 done")


if __name__ == "__main__":
    main()
