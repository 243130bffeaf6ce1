"""CPU fp32 restatement of TwoStream (TEST INFRASTRUCTURE ONLY — see oracle/__init__.py).

Parameters are a flat {state_dict name: tensor} dict with the reference's names:
  lang_model.*   HF BertModel names           (model/lang/bert_hugface.py:20)
  vision_model.* torchvision resnet50 names, TSM convs as `layerL.i.conv1.net.weight`
                 (ops/temporal_shift.py:21 wraps conv1 as `.net`)
  fusion_head.*  ChapterHead names            (model/fusion/two_stream.py:51-66)
"""
import math

import torch
import torch.nn.functional as F

STAGES = [(64, 3, 1), (128, 4, 2), (256, 6, 2), (512, 3, 2)]  # resnet50 (planes, blocks, stride)


def tsm_shift(x, n_segment, fold_div=8):
    """ops/temporal_shift.py:33-51 (out-of-place branch)."""
    nt, c, h, w = x.size()
    n_batch = nt // n_segment
    x = x.view(n_batch, n_segment, c, h, w)
    fold = c // fold_div
    out = torch.zeros_like(x)
    out[:, :-1, :fold] = x[:, 1:, :fold]
    out[:, 1:, fold:2 * fold] = x[:, :-1, fold:2 * fold]
    out[:, :, 2 * fold:] = x[:, :, 2 * fold:]
    return out.view(nt, c, h, w)


def _bn(p, name, y, mode, momentum=0.1, eps=1e-5):
    w, b = p[name + ".weight"], p[name + ".bias"]
    if mode == "running":
        return F.batch_norm(y, p[name + ".running_mean"], p[name + ".running_var"], w, b, False, momentum, eps)
    if mode == "train":  # batch statistics + in-place running-stat update
        return F.batch_norm(y, p[name + ".running_mean"], p[name + ".running_var"], w, b, True, momentum, eps)
    return F.batch_norm(y, None, None, w, b, True, momentum, eps)  # "batch": test driver semantics


def resnet50_tsm(p, x, n_segment, bn_mode, prefix="vision_model.", shift_div=8, tsm=True):
    """torchvision resnet50 (fc = Identity) with TemporalShift on each bottleneck conv1
    (make_temporal_shift blockres, temporal_shift.py:128-144). x [N,3,H,W] -> [N,2048].
    tsm=False: the plain torchvision resnet50 of model/vision/resnet50.py:9-73 (conv1 names without `.net`)."""
    y = F.conv2d(x, p[prefix + "conv1.weight"], stride=2, padding=3)
    y = F.relu(_bn(p, prefix + "bn1", y, bn_mode))
    y = F.max_pool2d(y, 3, 2, 1)
    for li, (planes, blocks, stride) in enumerate(STAGES):
        for bi in range(blocks):
            pre = f"{prefix}layer{li + 1}.{bi}."
            s = stride if bi == 0 else 1
            identity = y
            if tsm:
                out = F.conv2d(tsm_shift(y, n_segment, shift_div), p[pre + "conv1.net.weight"])
            else:
                out = F.conv2d(y, p[pre + "conv1.weight"])
            out = F.relu(_bn(p, pre + "bn1", out, bn_mode))
            out = F.conv2d(out, p[pre + "conv2.weight"], stride=s, padding=1)
            out = F.relu(_bn(p, pre + "bn2", out, bn_mode))
            out = F.conv2d(out, p[pre + "conv3.weight"])
            out = _bn(p, pre + "bn3", out, bn_mode)
            if bi == 0:
                identity = _bn(p, pre + "downsample.1", F.conv2d(y, p[pre + "downsample.0.weight"], stride=s),
                               bn_mode)
            y = F.relu(out + identity)
    return y.mean((2, 3))


def bert(p, ids, mask, prefix="lang_model.", n_layers=12, n_heads=12, eps=1e-12, p_drop=0.0, training=False):
    """HF BertModel eager forward (embeddings, 12 layers, tanh pooler) -> (pooled, last_hidden)."""
    B, L = ids.shape
    H = p[prefix + "embeddings.word_embeddings.weight"].shape[1]
    dh = H // n_heads
    pos = torch.arange(L)
    e = (p[prefix + "embeddings.word_embeddings.weight"][ids] + p[prefix + "embeddings.position_embeddings.weight"][pos]
         + p[prefix + "embeddings.token_type_embeddings.weight"][0])
    h = F.layer_norm(e, (H,), p[prefix + "embeddings.LayerNorm.weight"], p[prefix + "embeddings.LayerNorm.bias"], eps)
    h = F.dropout(h, p_drop, training)
    add = (1.0 - mask[:, None, None, :].float()) * torch.finfo(torch.float32).min
    for i in range(n_layers):
        pre = f"{prefix}encoder.layer.{i}."
        lin = lambda x, n: F.linear(x, p[pre + n + ".weight"], p[pre + n + ".bias"])  # noqa: E731
        q = lin(h, "attention.self.query").view(B, L, n_heads, dh).transpose(1, 2)
        k = lin(h, "attention.self.key").view(B, L, n_heads, dh).transpose(1, 2)
        v = lin(h, "attention.self.value").view(B, L, n_heads, dh).transpose(1, 2)
        s = q @ k.transpose(-1, -2) / math.sqrt(dh) + add
        a = F.dropout(torch.softmax(s, -1), p_drop, training)
        ctx = (a @ v).transpose(1, 2).reshape(B, L, H)
        ao = F.dropout(lin(ctx, "attention.output.dense"), p_drop, training)
        h1 = F.layer_norm(ao + h, (H,), p[pre + "attention.output.LayerNorm.weight"],
                          p[pre + "attention.output.LayerNorm.bias"], eps)
        ff = F.gelu(lin(h1, "intermediate.dense"))
        fo = F.dropout(lin(ff, "output.dense"), p_drop, training)
        h = F.layer_norm(fo + h1, (H,), p[pre + "output.LayerNorm.weight"], p[pre + "output.LayerNorm.bias"], eps)
    pooled = torch.tanh(F.linear(h[:, 0], p[prefix + "pooler.dense.weight"], p[prefix + "pooler.dense.bias"]))
    return pooled, h


def chapter_head_mlp(p, lang_emb, vision_emb, prefix="fusion_head."):
    """ChapterHead.forward (two_stream.py:71-95), head_type mlp."""
    B = lang_emb.shape[0]
    lang_out = F.relu(F.linear(lang_emb, p[prefix + "lang_proj_head.weight"])).unsqueeze(1)
    T = vision_emb.shape[1]
    vision_out = F.relu(F.linear(vision_emb.reshape(B * T, -1), p[prefix + "vision_proj_head.weight"])).view(B, T, -1)
    fusion = torch.cat([vision_out, lang_out], dim=1).view(B, -1)
    return F.linear(fusion, p[prefix + "head.weight"], p[prefix + "head.bias"])


def chapter_head_attn(p, lang_emb, vision_emb, n_head=4, prefix="fusion_head."):
    """ChapterHead.forward (two_stream.py:71-95), head_type attn: SelfAttention.forward (two_stream.py:31-48)
    over cat([vision_out, lang_out], 1) without dropout; output = proj of token 0."""
    B, T = vision_emb.shape[:2]
    lang_out = F.relu(F.linear(lang_emb, p[prefix + "lang_proj_head.weight"])).unsqueeze(1)
    vision_out = F.relu(F.linear(vision_emb.reshape(B * T, -1), p[prefix + "vision_proj_head.weight"])).view(B, T, -1)
    x = torch.cat([vision_out, lang_out], dim=1)
    C = x.shape[-1]
    hs = C // n_head

    def heads(name):
        y = F.linear(x, p[prefix + f"head.{name}.weight"], p[prefix + f"head.{name}.bias"])
        return y.view(B, T + 1, n_head, hs).transpose(1, 2)
    k, q, v = heads("key"), heads("query"), heads("value")
    att = torch.softmax((q @ k.transpose(-2, -1)) * (1.0 / math.sqrt(hs)), dim=-1)
    y = (att @ v).transpose(1, 2).contiguous().view(B, T + 1, C)
    return F.linear(y[:, 0, :], p[prefix + "head.proj.weight"], p[prefix + "head.proj.bias"])


def two_stream(p, img_clip, ids, mask, bn_mode="running", p_drop=0.0, training=False, head_type="mlp"):
    """TwoStream.forward (two_stream.py:172-194) -> logits, prob, vision_emb [B,T,2048], lang_emb."""
    B, T = img_clip.shape[:2]
    lang_emb, _ = bert(p, ids, mask, p_drop=p_drop, training=training)
    x = img_clip.reshape(B * T, *img_clip.shape[2:])
    vis = resnet50_tsm(p, x, T, bn_mode).view(B, T, -1)
    logits = (chapter_head_attn if head_type == "attn" else chapter_head_mlp)(p, lang_emb, vis)
    return logits, torch.softmax(logits, 1), vis, lang_emb


def linear_head(p, x, prefix="head."):
    """Single-model head: Linear + softmax (bert_hugface.py:124-126 on pooler_output, resnet50_tsm.py:68-77 on the
    [B, T*2048] concatenated frame embeddings)."""
    logits = F.linear(x, p[prefix + "weight"], p[prefix + "bias"])
    return logits, torch.softmax(logits, 1)


def param_groups(named, weight_decay):
    """TwoStream.configure_optimizers grouping (two_stream.py:135-164)."""
    decay, no_decay = [], []
    for n, t in named:
        pn = n.rsplit(".", 1)[-1]
        if pn.endswith("bias") or "LayerNorm" in n or "bn" in n or "emb" in n:
            no_decay.append((n, t))
        else:
            decay.append((n, t))
    decay.sort()
    no_decay.sort()
    return [{"params": [t for _, t in decay], "weight_decay": weight_decay},
            {"params": [t for _, t in no_decay], "weight_decay": 0.0}]


def train_step(params, buffers, img, ids, mask, labels, lr, betas=(0.9, 0.95), weight_decay=0.01, max_norm=1.0,
               head_type="mlp", p_drop=0.0):
    """One reference train step (train_video_segment_point.py:161-206 with accumulation 1):
    forward (BN train mode; BERT dropout p_drop in training mode, 0 by default: the parity fixtures) -> CE ->
    backward -> clip_grad_norm_ -> AdamW.step.
    params: {name: leaf tensor requiring grad}; buffers: {name: running stats} (updated in place)."""
    p = dict(buffers)
    p.update(params)
    logits, prob, _, _ = two_stream(p, img, ids, mask, bn_mode="train", head_type=head_type, p_drop=p_drop,
                                    training=p_drop > 0.0)
    loss = F.cross_entropy(logits, labels)
    loss.backward()
    total_norm = torch.nn.utils.clip_grad_norm_(list(params.values()), max_norm)
    opt = torch.optim.AdamW(param_groups(list(params.items()), weight_decay), lr=lr, betas=betas)
    opt.step()
    return loss.detach(), logits.detach(), total_norm.detach(), opt
