"""Parity of the bf16 train step that bench.py times (BASELINE config 3).

The bf16 trunk backward runs code the fp32 parity mode never touches: the fused conv_dgrad_bwd engine
(EPI_BWD / EPI_BWD_AFF epilogues: TSM adjoint, residual, ReLU mask, BN-backward sums), the sub-pixel
stride-2 class GEMMs, the dense stride-2 downsample input gradient (res_stride 2), the carried BN sums,
the pair-packed stem and wgrad_fast_kernel. These tests pin that path:

(a) C1 shapes (B=2, T=4, 112², L=32): the fused engine against the unfused bf16 ops on identical forward
    activations (every trunk gradient tensor), and the step's loss / logits against the exact fixture
    tests/golden/c1_train_fp64.npz (reference-run);
(b) Full resolution (B=2, T=16, 224², L=128): bf16 and fp32 native steps against the oracle's exact (fp64)
    gradients (oracle/model.py: CPU restatement of the reference, test infrastructure), next to the oracle's own
    fp32 (reference-arithmetic) gradients, on the same seeded weights and inputs.
(c) Full C3 (B=64, T=16, 224², L=128): finite, bit-identical across two runs, logits within bf16 tolerance of
    the fp32 native (train-mode) forward on the same inputs.

Tolerances (bf16 activations / MFMA operands, fp32 accumulation and statistics; the reference is fp32):
    loss within 1e-2; per-tensor relative Frobenius error <= 5e-2 for 95 % of tensors and <= 0.15 for all, cosine
    >= 0.995 for 95 % of tensors and >= 0.98 for all (BatchNorm over 8-32 frames amplifies bf16 rounding in the
    BN-adjacent parameter gradients); total gradient norm within 3e-2.
"""
import os
import re

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")
DEV = "cuda"


def _gold(name):
    return np.load(os.path.join(GOLD, name), allow_pickle=False)


class _Cfg:
    weight_decay = 0.01
    learning_rate = 1e-5
    betas = (0.9, 0.95)


def _model(T, precision, stats=None):
    from vcg_hip.build import build_two_stream
    return build_two_stream(clip_frame_num=T, seed=123, device=DEV, precision=precision, bn_stats=stats,
                            dropout=0.0).train()


def _step(model, frames, ids, mask, labels):
    """fwd + CE + bwd; returns (loss, logits, {name: grad (fp32, on the GPU)}, optimizer)."""
    from vcg_hip.functions import cross_entropy
    opt = model.configure_optimizers(_Cfg)
    opt.zero_grad()
    logits, _ = model(frames, ids, mask)
    loss = cross_entropy(logits, labels)
    loss.backward()
    torch.cuda.synchronize()
    grads = {n: p.grad.detach().clone() for n, p in model.named_parameters()}
    return loss.item(), logits.detach().float().cpu(), grads, opt


def _compare(ga, gb, tag):
    """per-tensor (rel Frobenius error of ga vs gb, cosine); gb is the reference."""
    out = {}
    for n in gb:
        a, b = ga[n].double().reshape(-1), gb[n].double().reshape(-1)
        nb = b.norm().item()
        if nb == 0.0:
            continue
        out[n] = ((a - b).norm().item() / nb, (a @ b).item() / max(a.norm().item() * nb, 1e-300))
    worst = sorted(out.items(), key=lambda kv: -kv[1][0])
    print(f"{tag}: rel-Frobenius / cosine per tensor, worst first:")
    for n, (e, c) in worst[:40]:
        print(f"   {n:70s} {e:.3e} {c:.6f} |ref| {gb[n].double().norm().item():.3e}")
    return out


def _check(stats, what):
    errs = np.array([e for e, _ in stats.values()])
    coss = np.array([c for _, c in stats.values()])
    assert np.isfinite(errs).all(), what
    assert np.quantile(errs, 0.95) <= 5e-2, f"{what}: 95th pct rel err {np.quantile(errs, 0.95):.3e}"
    assert errs.max() <= 0.15, f"{what}: max rel err {errs.max():.3e}"
    assert np.quantile(coss, 0.05) >= 0.995, f"{what}: 5th pct cosine {np.quantile(coss, 0.05):.5f}"
    assert coss.min() >= 0.98, f"{what}: min cosine {coss.min():.5f}"


def test_c1_bf16_fused_backward_vs_unfused():
    """The fused conv_dgrad_bwd engine against the unfused bf16 ops (conv_dgrad + bn_bwd_reduce / bn_bwd_apply +
    tsm_unshift_add) on IDENTICAL forward activations (the bf16 forward is deterministic and run twice): the
    backward is linear in the upstream gradient given the saved activations and masks, so the two differ only
    by bf16 rounding of the intermediate gradients -- no forward-difference amplification through the BatchNorm
    statistics (see test_c1_loss_and_conditioning). C1 shapes; every trunk parameter gradient compared."""
    from vcg_hip import synth
    from vcg_hip.trunk import ResNetTrunk
    st = dict(_gold("bn_running_stats.npz"))
    frames, ids, mask, labels = synth.clip_batch(2, 4, 112, 112, 32, seed=123, device=DEV)
    m = _model(4, "bf16", st)
    saved = ResNetTrunk.gram_stats
    try:
        # (bn3's statistics from the conv3 GEMM in both runs: the unfused path has no Gram pass, and this comparison
        # needs the same forward -- test_gram_stats_forward covers the Gram statistics)
        ResNetTrunk.gram_stats = False
        ResNetTrunk.fused_bwd = False
        lu, lgu, gu, _ = _step(m, frames, ids, mask, labels)
        ResNetTrunk.fused_bwd = True
        lf, lgf, gf, _ = _step(m, frames, ids, mask, labels)
    finally:
        ResNetTrunk.fused_bwd = True
        ResNetTrunk.gram_stats = saved
    assert lu == lf and torch.equal(lgu, lgf), "the forward is not deterministic"
    stats = _compare({n: v for n, v in gf.items() if n.startswith("vision_model")},
                     {n: v for n, v in gu.items() if n.startswith("vision_model")}, "C1 bf16 fused vs unfused")
    errs = np.array([e for e, _ in stats.values()])
    coss = np.array([c for _, c in stats.values()])
    print(f"fused vs unfused: rel err median {np.median(errs):.2e} max {errs.max():.2e}; cosine min {coss.min():.6f}")
    # two bf16 rounding orders of the same linear backward: ~1e-2 (measured: median 1.2e-2, max 4.9e-2 on
    # vision_model.bn1.bias, cosine >= 0.9988)
    assert np.median(errs) <= 2e-2 and errs.max() <= 8e-2 and coss.min() >= 0.998
    for n in gf:  # BERT and the head run identical code in both passes
        if not n.startswith("vision_model"):
            assert torch.equal(gf[n], gu[n]), n


def test_c1_bf16_bn_fold_vs_apply():
    """bn3's batch-statistics backward folded into conv3's input / weight gradients (VCG_BN_FOLD, no dy3 tensor)
    against the bn_bwd_apply pass, same forward: two bf16 rounding orders of the same linear backward (the fold
    rounds A w / B w, the pass rounds dy3), held to the fused-vs-unfused bounds; both runs deterministic."""
    from vcg_hip import synth
    from vcg_hip.trunk import ResNetTrunk
    st = dict(_gold("bn_running_stats.npz"))
    frames, ids, mask, labels = synth.clip_batch(2, 4, 112, 112, 32, seed=123, device=DEV)
    m = _model(4, "bf16", st)
    saved = ResNetTrunk.bn_fold_bwd, ResNetTrunk.gram_stats
    try:
        # (bn3's statistics from the conv3 GEMM in both runs: the Gram statistics of the fold's forward are not
        # bit-identical to them, and this comparison needs the same forward -- test_gram_stats_forward covers them)
        ResNetTrunk.gram_stats = False
        ResNetTrunk.bn_fold_bwd = False
        la, lga, ga, _ = _step(m, frames, ids, mask, labels)
        ResNetTrunk.bn_fold_bwd = True
        ResNetTrunk.path_counts = {"fused": 0, "unfused": 0}
        lb, lgb, gb, _ = _step(m, frames, ids, mask, labels)
        assert ResNetTrunk.path_counts["unfused"] == 0
        lc, lgc, gc, _ = _step(m, frames, ids, mask, labels)
    finally:
        ResNetTrunk.bn_fold_bwd, ResNetTrunk.gram_stats = saved
    assert la == lb == lc and torch.equal(lga, lgb)
    for n in gb:
        assert torch.equal(gb[n], gc[n]), n
    stats = _compare({n: v for n, v in gb.items() if n.startswith("vision_model")},
                     {n: v for n, v in ga.items() if n.startswith("vision_model")}, "C1 bf16 bn3 fold vs apply")
    errs = np.array([e for e, _ in stats.values()])
    coss = np.array([c for _, c in stats.values()])
    print(f"fold vs apply: rel err median {np.median(errs):.2e} max {errs.max():.2e}; cosine min {coss.min():.6f}")
    assert np.median(errs) <= 2e-2 and errs.max() <= 8e-2 and coss.min() >= 0.998


def test_gram_fin_model_identical():
    """The fused bn3 statistics + finalize + weight fold launch (ResNetTrunk.gram_fin) against the three-call chain in
    a whole bf16 train step: bit-identical loss, gradients and BN running statistics."""
    from vcg_hip import synth
    from vcg_hip.trunk import ResNetTrunk
    st = dict(_gold("bn_running_stats.npz"))
    frames, ids, mask, labels = synth.clip_batch(2, 4, 112, 112, 32, seed=78, device=DEV)
    res = {}
    saved = ResNetTrunk.gram_fin
    try:
        for fin in (True, False):
            ResNetTrunk.gram_fin = fin
            m = _model(4, "bf16", st)
            loss, _, g, _ = _step(m, frames, ids, mask, labels)
            run = {n: b.detach().clone() for n, b in m.named_buffers() if "running" in n}
            res[fin] = (loss, g, run)
    finally:
        ResNetTrunk.gram_fin = saved
    (l1, g1, r1), (l2, g2, r2) = res[True], res[False]
    assert l1 == l2
    assert g1.keys() == g2.keys() and all(torch.equal(g1[n], g2[n]) for n in g1)
    assert r1.keys() == r2.keys() and len(r1) > 0 and all(torch.equal(r1[n], r2[n]) for n in r1)


def test_gram_stats_forward():
    """bn3's batch statistics from the bn2 apply pass's (a2^T a2, colsum(a2)) (ResNetTrunk.gram_stats, the exact y3
    statistics) against the conv3 statistics GEMM (of the bf16-rounded y3), C1 shapes, BN in training mode: the
    bf16 train forward's vision embeddings and logits sit as close to the fp32 native forward with either (rel. error
    no worse than 1.25 x + 2e-3 / logits 1.25 x + 1e-2), and the Gram path's backward is deterministic and finite."""
    from vcg_hip import synth
    from vcg_hip.trunk import ResNetTrunk
    st = dict(_gold("bn_running_stats.npz"))
    frames, ids, mask, labels = synth.clip_batch(2, 4, 112, 112, 32, seed=77, device=DEV)
    res = {}
    saved = ResNetTrunk.gram_stats
    try:
        for tag, prec, gram in (("gram", "bf16", True), ("gemm", "bf16", False), ("fp32", "fp32", False)):
            ResNetTrunk.gram_stats = gram
            m = _model(4, prec, st)
            lg, _, ve, _ = m(frames, ids, mask, return_emb=True)
            res[tag] = (lg.detach().double().cpu(), ve.detach().double().cpu())
            if tag == "gram":
                l1, _, g1, _ = _step(m, frames, ids, mask, labels)
                l2, _, g2, _ = _step(m, frames, ids, mask, labels)
                assert l1 == l2 and all(torch.equal(g1[n], g2[n]) for n in g1)
                assert all(torch.isfinite(v).all() for v in g1.values())
    finally:
        ResNetTrunk.gram_stats = saved
    lg32, ve32 = res["fp32"]
    e = {t: (_rel(res[t][1], ve32), (res[t][0] - lg32).abs().max().item()) for t in ("gram", "gemm")}
    print("vision emb rel err / logits max err vs fp32:", e)
    assert e["gram"][0] <= 1.25 * e["gemm"][0] + 2e-3
    assert e["gram"][1] <= 1.25 * e["gemm"][1] + 1e-2


@pytest.mark.parametrize("prec", ["fp32", "bf16"])
def test_pooled_stem_sums_step(prec):
    """The stem backward variants -- BN-backward sums from the pooled activation (ResNetTrunk.pooled_stem_sums) and
    the one-pass apply + conv1 weight gradient (ResNetTrunk.fused_stem_bwd, bf16 only) -- against the per-pixel sums
    pass, the dy0 apply pass and the im2col weight gradient, one C1-shape train step: the same loss; gradients the
    same up to the rounding of the recovered activation and the summation order (fp32: every tensor within 1e-4
    relative; bf16: the stem conv / BN gradients, the only ones these reach, within 2e-2 relative, cosine >=
    0.999)."""
    from vcg_hip import synth
    from vcg_hip.trunk import ResNetTrunk
    st = dict(_gold("bn_running_stats.npz"))
    frames, ids, mask, labels = synth.clip_batch(2, 4, 112, 112, 32, seed=78, device=DEV)
    res = {}
    saved = ResNetTrunk.pooled_stem_sums, ResNetTrunk.fused_stem_bwd
    try:
        for new in (True, False):
            ResNetTrunk.pooled_stem_sums = ResNetTrunk.fused_stem_bwd = new
            res[new] = _step(_model(4, prec, st), frames, ids, mask, labels)
    finally:
        ResNetTrunk.pooled_stem_sums, ResNetTrunk.fused_stem_bwd = saved
    (la, _, ga, _), (lb, _, gb, _) = res[True], res[False]
    assert la == lb
    for n in gb:
        e = _rel(ga[n].cpu(), gb[n].double().cpu())
        if prec == "fp32":
            assert e <= 1e-4, (n, e)
        elif e > 2e-2:
            raise AssertionError((n, e))
        x, y = ga[n].double().flatten(), gb[n].double().flatten()
        if y.norm().item() > 0:  # (explicit: torch's cosine_similarity clamps norms below 1e-8)
            cos = (x @ y).item() / max(x.norm().item() * y.norm().item(), 1e-300)
            assert cos >= 0.999, (n, cos)


@pytest.mark.parametrize("wgrad_stream,ds_stream", [(True, False), (False, False), (False, True)])
def test_side_stream_settings_identical(wgrad_stream, ds_stream):
    """The trunk backward's side-stream settings change where kernels run, never what they compute: with the
    weight-gradient stream on and the downsample stream off (the downsample BN's backward apply then runs inline,
    because conv1's fused dgrad on the main stream reads its dyd) and the other combinations, one C1-shape bf16
    train step gives bit-identical loss and gradients to the default (both side streams on)."""
    from vcg_hip import synth
    from vcg_hip.trunk import ResNetTrunk
    frames, ids, mask, labels = synth.clip_batch(2, 4, 112, 112, 32, seed=17, device=DEV)
    saved = ResNetTrunk.wgrad_stream, ResNetTrunk.ds_stream
    res = {}
    try:
        for tag, (wg, ds) in (("default", (True, True)), ("alt", (wgrad_stream, ds_stream))):
            ResNetTrunk.wgrad_stream, ResNetTrunk.ds_stream = wg, ds
            m = _model(4, "bf16")
            res[tag] = _step(m, frames, ids, mask, labels)
            del m
    finally:
        ResNetTrunk.wgrad_stream, ResNetTrunk.ds_stream = saved
    (la, lga, ga, _), (lb, lgb, gb, _) = res["default"], res["alt"]
    assert la == lb and torch.equal(lga, lgb)
    diff = [n for n in ga if not torch.equal(ga[n], gb[n])]
    assert not diff, f"gradients differ with wgrad_stream={wgrad_stream} ds_stream={ds_stream}: {diff[:6]}"


def test_c1_loss_and_conditioning():
    """C1 bf16 step: loss / logits within bf16 tolerance of the exact fixture. (Its vision gradients are NOT
    compared element-wise with fp32: at C1 the BatchNorm statistics run over 8 frames of 4x4..56x56 maps and the
    reference's OWN fp32 gradients already deviate from fp64 by up to 4 % on BN-adjacent tensors -- an
    amplification of ~1e5 of fp32 rounding; bf16 rounding (4e-3) saturates it. The fused kernels are pinned by
    test_c1_bf16_fused_backward_vs_unfused, the end-to-end step at full resolution by
    test_full_res_train_step_vs_oracle.)"""
    from vcg_hip import synth
    st = dict(_gold("bn_running_stats.npz"))
    g = _gold("c1_train.npz")
    g64 = _gold("c1_train_fp64.npz")
    frames, ids, mask, labels = synth.clip_batch(2, 4, 112, 112, 32, seed=123, device=DEV)
    m16 = _model(4, "bf16", st)
    l16, lg16, g16, _ = _step(m16, frames, ids, mask, labels)
    print(f"C1 loss bf16 {l16:.6f} exact {float(g64['loss'][0]):.6f}")
    assert abs(l16 - float(g64["loss"][0])) < 1e-2
    assert (lg16 - torch.from_numpy(g["train_logits"])).abs().max().item() < 5e-2
    for n, v in g16.items():
        assert torch.isfinite(v).all(), n


def test_c1_bf16_census():
    """The bf16 step runs the fused engines: no unfused dgrad fallback, fast GEMM and fast wgrad launches."""
    from vcg_hip import synth
    frames, ids, mask, labels = synth.clip_batch(2, 4, 112, 112, 32, seed=5, device=DEV)
    m16 = _model(4, "bf16")
    from vcg_hip import ops
    from vcg_hip.functions import cross_entropy
    from vcg_hip.trunk import ResNetTrunk
    ResNetTrunk.path_counts.update(fused=0, unfused=0)
    ops.timing_enable(True)
    loss = cross_entropy(m16(frames, ids, mask)[0], labels)
    loss.backward()
    torch.cuda.synchronize()
    n_fast = ops.timing_query(ops.TIMING_FAST_GEMM)[1]
    n_wg = ops.timing_query(ops.TIMING_WGRAD)[1]
    ops.timing_enable(False)
    cen = dict(ResNetTrunk.path_counts)
    print("census", cen, "fast_gemm launches", n_fast, "wgrad_fast launches", n_wg)
    assert cen["unfused"] == 0 and cen["fused"] == 2 * 16 + 16  # conv2 + conv3 dgrad per block, conv1 dgrad per block
    assert n_fast > 0 and n_wg > 0


def _oracle_step(T, HW, L, B, seed, dtype=torch.float32, autocast=False):
    """oracle.model two_stream forward (BN train mode) + CE + backward on the CPU, in fp32 (the reference's
    arithmetic), fp64 (exact) or fp32 under torch.autocast(bf16) (the reference's arithmetic in bf16, as
    PyTorch would run it): (loss, logits, vision_emb, {name: grad}) -- the gradients oracle.model.train_step clips
    and steps with."""
    from oracle import model as om
    from vcg_hip import synth
    from vcg_hip.build import build_two_stream
    torch.set_num_threads(min(16, len(os.sched_getaffinity(0))))
    m = build_two_stream(clip_frame_num=T, seed=123, dropout=0.0)
    sd = m.state_dict()
    names = [n for n, _ in m.named_parameters()]
    params = {n: sd[n].detach().to(dtype).clone().requires_grad_() for n in names}
    buffers = {n: (sd[n].detach().to(dtype).clone() if sd[n].is_floating_point() else sd[n]) for n in sd
               if n not in params}
    frames, ids, mask, labels = synth.clip_batch(B, T, HW, HW, L, seed=seed)
    p = dict(buffers)
    p.update(params)
    with torch.autocast("cpu", dtype=torch.bfloat16, enabled=autocast):
        logits, _, vis, _ = om.two_stream(p, frames.to(dtype), ids, mask, bn_mode="train")
        loss = torch.nn.functional.cross_entropy(logits.float(), labels)
    loss.backward()
    return loss.item(), logits.detach().double(), vis.detach().double(), {n: params[n].grad.double() for n in names}


def _rel(a, b):
    return (a.double() - b).norm().item() / max(b.norm().item(), 1e-300)


def test_full_res_train_step_vs_oracle():
    """B=1, T=16, 224², L=128 (the C3 window shape), one train step with BatchNorm batch statistics. (One window:
    with B >= 2 the head / BERT gradients of a random-init model are dominated by the small DIFFERENCES between
    the windows' nearly identical features, which amplifies any rounding -- torch autocast's own BERT gradients are
    4 % off exact at B=2 and 1.7 % at B=1, its head gradients 21 % vs 6 %.)

    fp32 native: loss within 1e-4, logits within 1e-3 of the exact (fp64) oracle, and every gradient tensor as
    close to exact as the reference-arithmetic fp32 oracle is (|ours - f64| <= max(3 |ref32 - f64|, 2e-3)).

    bf16 native (the benchmarked path) against the same reference arithmetic run in bf16 by PyTorch
    (torch.autocast on the CPU oracle): at random init this network is exponentially sensitive to rounding
    (batch-stat BatchNorm through 16 bottlenecks: the fp32 oracle's own vision gradients are ~2 % off exact,
    bf16 autocast's ~100 %, its vision embeddings ~13 %), so the bf16 step is held to PyTorch-bf16's accuracy:
    logits / vision embeddings / every gradient group within 1.5x of autocast's error vs exact (+ a small floor),
    loss within 1e-2; BERT's gradients within 1.5 x autocast's error of exact (median and 90th percentile over its
    tensors, no floor).

    Kernel census: the GEMM kernels this B = 1 step ran (vcg_gemm_census, every GEMM-class launch) are the kernels a
    B = 64 step (the bench's C3 configuration) runs -- kernel selection does not depend on the batch, so this
    oracle-anchored step exercises the benchmarked GEMM path (BERT's Linear layers on the wide-tile engine, the layer-4
    3x3 forward convs on the 256-tile engine, ...)."""
    from vcg_hip import ops, synth
    B, T, HW, L = 1, 16, 224, 128
    l64, lg64, v64, g64 = _oracle_step(T, HW, L, B, seed=11, dtype=torch.float64)
    lo, lgo, vo, go = _oracle_step(T, HW, L, B, seed=11)
    la, lga, va, ga = _oracle_step(T, HW, L, B, seed=11, autocast=True)
    frames, ids, mask, labels = synth.clip_batch(B, T, HW, HW, L, seed=11, device=DEV)
    from vcg_hip.trunk import ResNetTrunk
    res = {}
    for prec in ("fp32", "bf16"):
        m = _model(T, prec)
        from vcg_hip.functions import cross_entropy
        opt = m.configure_optimizers(_Cfg)
        opt.zero_grad()
        ResNetTrunk.census = [] if prec == "bf16" else None
        ops.gemm_census_enable(prec == "bf16")
        try:
            lg, _, ve, _ = m(frames, ids, mask, return_emb=True)
            loss = cross_entropy(lg, labels)
            loss.backward()
            torch.cuda.synchronize()
            census = ResNetTrunk.census
            gemms = ops.gemm_census()
        finally:
            ResNetTrunk.census = None
            ops.gemm_census_enable(False)
        if prec == "bf16":  # the oracle-anchored bf16 step ran the benchmarked per-block paths
            _check_census(census)
            anchored_kernels = _gemm_kernels(gemms)
            # (BERT's rows: B * L, or fewer where its padded rows are dropped -- BertEncoderEngine.unpad)
            bert_wide = [k for k in gemms if k.startswith("gemm_wide") and any(f" N={n} " in k for n in (768, 2304, 3072))]
            assert len(bert_wide) >= 4, gemms  # QKV / out-proj / FFN1 / FFN2 forward and their input gradients
        res[prec] = (loss.item(), lg.detach().double().cpu(), ve.detach().double().cpu(),
                     {n: p.grad.detach().double().cpu() for n, p in m.named_parameters()})
        del m, opt
        torch.cuda.empty_cache()
    bench_kernels = _bench_step_kernels(T, HW, L)
    print("GEMM kernels, B=1 step:", sorted(anchored_kernels))
    assert bench_kernels == anchored_kernels, ("the B=64 step runs kernels the anchored step does not",
                                               sorted(bench_kernels ^ anchored_kernels))
    l32, lg32, v32, g32 = res["fp32"]
    l16, lg16, v16, g16 = res["bf16"]
    print(f"loss exact {l64:.6f} oracle32 {lo:.6f} autocast-bf16 {la:.6f} native fp32 {l32:.6f} bf16 {l16:.6f}")
    print(f"vision_emb rel err vs exact: oracle32 {_rel(vo, v64):.2e} autocast {_rel(va, v64):.2e} "
          f"native fp32 {_rel(v32, v64):.2e} bf16 {_rel(v16, v64):.2e}")
    print(f"logits max err vs exact: autocast {(lga - lg64).abs().max().item():.3e} bf16 {(lg16 - lg64).abs().max().item():.3e}")
    gmax = max(v.norm().item() for v in g64.values())
    keep = [n for n, v in g64.items() if v.norm().item() > 1e-6 * gmax]  # key.bias: analytically zero
    # fp32 native
    assert abs(l32 - l64) < 1e-4 and (lg32 - lg64).abs().max().item() < 1e-3
    bad = [(n, _rel(g32[n], g64[n]), _rel(go[n], g64[n])) for n in keep
           if _rel(g32[n], g64[n]) > max(3 * _rel(go[n], g64[n]), 2e-3)]
    assert not bad, f"fp32 native gradients off: {bad[:6]}"
    # bf16 native vs PyTorch-bf16 accuracy
    assert abs(l16 - l64) < 1e-2
    assert _rel(v16, v64) <= 1.5 * _rel(va, v64) + 1e-2
    assert (lg16 - lg64).abs().max().item() <= 1.5 * (lga - lg64).abs().max().item() + 1e-2
    for group in ("vision_model", "lang_model", "fusion_head"):
        names = [n for n in keep if n.startswith(group)]
        e16 = np.array([_rel(g16[n], g64[n]) for n in names])
        eac = np.array([_rel(ga[n], g64[n]) for n in names])
        print(f"{group}: grad rel err vs exact median / p90: native bf16 {np.median(e16):.2e} / "
              f"{np.quantile(e16, 0.9):.2e}, autocast bf16 {np.median(eac):.2e} / {np.quantile(eac, 0.9):.2e}")
        worst = sorted(zip(e16, eac, names), key=lambda t: -t[0])[:10]
        print(f"{group} worst:", [(n.split(".", 1)[1][-40:], f"{a:.2e}", f"{b:.2e}") for a, b, n in worst])
        floor = {"vision_model": 1e-2, "lang_model": 0.0, "fusion_head": 5e-2}[group]
        assert np.median(e16) <= max(1.5 * np.median(eac), floor), group
        assert np.quantile(e16, 0.9) <= max(1.5 * np.quantile(eac, 0.9), 2 * floor), group


def _gemm_kernels(gemms):
    """The GEMM kernels (census keys without shape and split count) of a step."""
    return {re.sub(r" z\d+", "", k.split(" M=")[0]) for k in gemms}


def _bench_step_kernels(T, HW, L, B=64):
    """GEMM kernels of one bf16 train step at the bench's C3 configuration (B = 64 windows)."""
    from vcg_hip import ops, synth
    from vcg_hip.functions import cross_entropy
    frames, ids, mask, labels = synth.clip_batch(B, T, HW, HW, L, seed=5, device=DEV)
    m = _model(T, "bf16")
    ops.gemm_census_enable(True)
    try:
        loss = cross_entropy(m(frames, ids, mask)[0], labels)
        loss.backward()
        torch.cuda.synchronize()
        gemms = ops.gemm_census()
    finally:
        ops.gemm_census_enable(False)
    del m, frames, loss
    torch.cuda.empty_cache()
    return _gemm_kernels(gemms)


def _check_census(census):
    """Per block, at the C3 shape, which of the round-3 bn3 paths engaged (the eligibility predicates fall back
    silently, so the benchmarked configuration is asserted block by block): layers 1-3 (C3 <= 1024) fold bn3's
    backward into conv3's two gradients in the a2 form (colsum(a2) from the bn2 apply pass); their non-first blocks
    also drop y3 (statistics-only conv3) and apply bn3 + residual + ReLU as a second conv3 GEMM pass; layer 4
    (C3 = 2048) runs the bn_apply / bn_bwd_apply passes."""
    fwd = [c for c in census if c[0] == "fwd"]
    bwd = [c for c in census if c[0] == "bwd"][::-1]  # (the backward walks the blocks in reverse)
    assert len(fwd) == 16 and len(bwd) == 16, (len(fwd), len(bwd))
    for i, ((_, c3, ds, f), (_, c3b, dsb, b)) in enumerate(zip(fwd, bwd)):
        assert (c3, ds) == (c3b, dsb)
        small = c3 <= 1024
        want_f = {"a2sum": small, "y3_drop": small and not ds, "bn3_gemm": small and not ds}
        # P = g^T a2 from the next block's streaming conv1 dgrad: layer-1 blocks 1-2
        want_b = {"fold_wgrad": small, "fold_dgrad": small, "p_dgrad": i in (1, 2), "a2_form": small}
        assert f == want_f, (c3, ds, f)
        assert b == want_b, (c3, ds, b)


def test_c3_bf16_train_step_properties():
    """Full C3 (B=64): finite, bit-identical across runs, logits close to the fp32 native train-mode forward; the
    per-block bn3 paths of the benchmarked configuration engaged (_check_census)."""
    from vcg_hip import synth
    B, T, HW, L = 64, 16, 224, 128
    frames, ids, mask, labels = synth.clip_batch(B, T, HW, HW, L, seed=123, device=DEV)
    from vcg_hip.trunk import ResNetTrunk
    runs = []
    for it in range(2):
        m = _model(T, "bf16")
        ResNetTrunk.census = [] if it == 0 else None
        try:
            loss, lg, gr, opt = _step(m, frames, ids, mask, labels)
            census = ResNetTrunk.census
        finally:
            ResNetTrunk.census = None
        if it == 0:
            _check_census(census)
        assert np.isfinite(loss) and torch.isfinite(lg).all()
        assert all(torch.isfinite(v).all().item() for v in gr.values())
        runs.append((loss, lg, gr))
        del m, opt
    (la, lga, ga), (lb, lgb, gb) = runs
    assert la == lb and torch.equal(lga, lgb)
    diff = [n for n in ga if not torch.equal(ga[n], gb[n])]
    assert not diff, f"non-deterministic gradients: {diff[:5]}"
    del runs, gb
    torch.cuda.empty_cache()
    m32 = _model(T, "fp32")
    with torch.no_grad():
        lg32, _ = m32(frames, ids, mask)  # train-mode forward (batch statistics), same inputs
    d = (lga - lg32.float().cpu()).abs().max().item()
    print(f"C3 logits bf16 vs fp32: max diff {d:.3e}")
    assert d <= 5e-2


def test_eval_bn3_fold_matches_unfolded():
    """The bf16 scoring forward (running-statistics BN, no autograd) folds every bottleneck BN into the conv before it
    (vcg_weight_fold; conv1 / conv2 / downsample via vcg_conv_fwd_bias_act, conv3 as one GEMM with bias, residual and
    ReLU; trunk._block_fwd_folded). Against the unfolded bf16 forward (conv -> y -> bn_apply) and the fp32 parity
    forward on the same weights, reference-run running statistics and inputs: the
    vision embeddings of both bf16 paths sit equally close to fp32 (rel. Frobenius error no worse than 1.25 x the
    unfolded path's + 2e-3; both ~0.15 here: the reference-run statistics do not match random-init activations, and
    eval BN amplifies bf16 rounding), and the folded logits no further from fp32 than 1.25 x the unfolded ones + 1e-2."""
    from vcg_hip import synth
    from vcg_hip.trunk import ResNetTrunk
    st = dict(_gold("bn_running_stats.npz"))
    frames, ids, mask, _ = synth.clip_batch(4, 4, 112, 112, 32, seed=321, device=DEV)
    res = {}
    saved = ResNetTrunk.fold_eval
    try:
        for tag, prec, fold in (("fold", "bf16", True), ("plain", "bf16", False), ("fp32", "fp32", False)):
            ResNetTrunk.fold_eval = fold
            m = _model(4, prec, st).eval()
            with torch.no_grad():
                logits, _, vis, _ = m(frames, ids, mask, return_emb=True)
            torch.cuda.synchronize()
            res[tag] = (logits.float().cpu().double(), vis.float().cpu().double())
    finally:
        ResNetTrunk.fold_eval = saved
    ref = res["fp32"][1]
    ef = ((res["fold"][1] - ref).norm() / ref.norm()).item()
    ep = ((res["plain"][1] - ref).norm() / ref.norm()).item()
    print(f"vision emb vs fp32: folded {ef:.3e}, unfolded {ep:.3e}")
    assert torch.isfinite(res["fold"][1]).all()
    assert ef <= 1.25 * ep + 2e-3, (ef, ep)
    lf = (res["fold"][0] - res["fp32"][0]).abs().max().item()
    lp = (res["plain"][0] - res["fp32"][0]).abs().max().item()
    print(f"logits vs fp32: folded {lf:.3e}, unfolded {lp:.3e}")
    assert lf <= 1.25 * lp + 1e-2, (lf, lp)
