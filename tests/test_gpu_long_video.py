"""Config 5 (long-video inference) on the GPU: window gather + normalisation on the device
(vcg_window_frames_u8), TwoStream scoring through forward_staged, boundary metrics -- against the CPU oracle
(oracle/model.py, pinned by the reference goldens) on the same synthetic video and windows.

Tolerance: fp32 parity mode, prob[:, 1] within 1e-3; predicted labels identical wherever the oracle's
probability is more than 1e-3 away from the 0.5 decision boundary; boundary metrics identical when all labels
agree."""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")
DEV = "cuda"


def test_long_video_pipeline_matches_oracle():
    import long_video as lv
    from data.synthetic_dataset import HashTokenizer, normalize_frames
    from oracle import model as om
    from vcg_hip.build import build_two_stream
    stats = dict(np.load(os.path.join(GOLD, "bn_running_stats.npz"), allow_pickle=False))
    F, T, HW, L = 40, 4, 112, 32
    model = build_two_stream(clip_frame_num=T, seed=123, device=DEV, precision="fp32", bn_stats=stats,
                             dropout=0.0).eval()
    frames, timestamps, subtitles = lv.synthetic_long_video(F, HW, HW, chapter_every=12, seed=5, device=DEV)
    win, idx, ids, mask = lv.window_inputs(F, T, 1, subtitles, HashTokenizer(), L)
    assert len(win) == F - T
    assert np.array_equal(idx[:, 0], np.where((win[:, 0] <= 2) | (win[:, 0] >= F - T - 2), win[:, 0], win[:, 0] + 2))
    scores, labels = lv.score_windows(model, frames, torch.from_numpy(idx).to(DEV), torch.from_numpy(ids).to(DEV),
                                      torch.from_numpy(mask).to(DEV), batch_size=16)
    torch.cuda.synchronize()
    p = {k: v.detach().cpu() for k, v in model.state_dict().items()}
    img = normalize_frames(frames.cpu().numpy()[idx])  # [n, T, 3, H, W]
    with torch.no_grad():
        _, pr, _, _ = om.two_stream(p, img, torch.from_numpy(ids), torch.from_numpy(mask), bn_mode="running")
    ref = pr[:, 1].numpy()
    got = scores.cpu().numpy()
    assert np.abs(got - ref).max() < 1e-3, np.abs(got - ref).max()
    ref_lab = (pr[:, 1] > pr[:, 0]).long().numpy()
    sure = np.abs(ref - 0.5) > 1e-3
    assert np.array_equal(labels.cpu().numpy()[sure], ref_lab[sure])
    if np.array_equal(labels.cpu().numpy(), ref_lab):
        assert lv.boundary_metrics(labels.cpu().tolist(), timestamps, F, T, 1) == \
            lv.boundary_metrics(ref_lab.tolist(), timestamps, F, T, 1)


def test_long_video_bf16_runs_and_exports(tmp_path):
    """The throughput configuration (bf16, vision-embedding export of convert2vision_emb): every window is
    scored, the exported [T, 2048] embeddings equal the ones the forward returns."""
    import long_video as lv
    from convert2vision_emb import load_vision_emb
    from data.synthetic_dataset import HashTokenizer
    from vcg_hip.build import build_two_stream
    F, T, HW, L = 30, 4, 112, 32
    model = build_two_stream(clip_frame_num=T, seed=123, device=DEV, precision="bf16").eval()
    frames, timestamps, subtitles = lv.synthetic_long_video(F, HW, HW, chapter_every=10, seed=6, device=DEV)
    win, idx, ids, mask = lv.window_inputs(F, T, 1, subtitles, HashTokenizer(), L)
    saved = {}

    def export(b0, ve):
        for k in range(ve.shape[0]):
            saved[b0 + k] = ve[k].float().cpu().numpy()
            s, e = win[b0 + k]
            d = os.path.join(tmp_path, "v")
            os.makedirs(d, exist_ok=True)
            np.save(os.path.join(d, f"vision_emb_{int(s)}_{int(e)}.npy"), saved[b0 + k])
    scores, labels = lv.score_windows(model, frames, torch.from_numpy(idx).to(DEV), torch.from_numpy(ids).to(DEV),
                                      torch.from_numpy(mask).to(DEV), batch_size=8, export=export)
    torch.cuda.synchronize()
    assert len(saved) == len(win) and torch.isfinite(scores).all()
    s, e = win[3]
    assert np.array_equal(load_vision_emb(str(tmp_path), "v", int(s), int(e)), saved[3])
    m = lv.boundary_metrics(labels.cpu().tolist(), timestamps, F, T, 1)
    assert m["gt_cut_points"] and 0.0 <= m["recall"] <= 1.0


def test_c5_full_size_bf16_vs_fp32_and_oracle():
    """BASELINE config 5 at its configured size: a 3600-frame (1 h @ 1 fps) 224² video, T=16, L=128, stride-1 s
    windows (3584 of them), running-stat BN (eval). Every window is scored by the benchmarked bf16 path and by the
    fp32 parity mode; 16 windows spread over the video are checked against the CPU oracle (fp32, 1e-3).

    The random-init head is re-biased (fusion_head.head.bias, from a 256-window fp32 sample) so that about half the
    windows are positive -- otherwise every window lands on one side of 0.5 and the label / F1 comparison is empty.
    bf16 vs fp32: prob[:, 1] within 5e-2 everywhere; labels may differ only on windows whose fp32 probability is
    within 5 x the median |p_bf16 - p_fp32| of the 0.5 boundary; the boundary metrics of both are reported and the
    F scores must agree within the share of flipped windows."""
    import long_video as lv
    from data.synthetic_dataset import HashTokenizer, normalize_frames
    from oracle import model as om
    from vcg_hip import ops
    from vcg_hip.build import build_two_stream
    stats = dict(np.load(os.path.join(GOLD, "bn_running_stats.npz"), allow_pickle=False))
    F, T, HW, L, S = 3600, 16, 224, 128, 1
    frames, timestamps, subtitles = lv.synthetic_long_video(F, HW, HW, seed=123, device=DEV)
    win, idx, ids, mask = lv.window_inputs(F, T, S, subtitles, HashTokenizer(), L)
    assert len(win) == 3584
    idx_d, ids_d, mask_d = (torch.from_numpy(a).to(DEV) for a in (idx, ids, mask))
    models = {p: build_two_stream(clip_frame_num=T, seed=123, device=DEV, precision=p, bn_stats=stats,
                                  dropout=0.0).eval() for p in ("fp32", "bf16")}
    # re-bias the 2-way head so the decisions split: shift logit 1 by the median margin of a sample
    samp = np.linspace(0, len(win) - 1, 256).astype(np.int64)
    with torch.no_grad():
        fr = ops.window_frames_u8(frames, idx_d[samp].contiguous(), torch.float32, cpad=ops.stem_cpad(torch.float32))
        lg, _ = models["fp32"].forward_staged(fr, ids_d[samp], mask_d[samp])
        shift = (lg[:, 0] - lg[:, 1]).median().item()
        for m in models.values():
            m.fusion_head.head.bias.data[1] += shift
            m.native_flat().refresh_shadow(force=True)
    res = {}
    for p, m in models.items():
        sc, lab = lv.score_windows(m, frames, idx_d, ids_d, mask_d, batch_size=64)
        torch.cuda.synchronize()
        res[p] = (sc.cpu().numpy().astype(np.float64), lab.cpu().numpy())
    p32, l32 = res["fp32"]
    p16, l16 = res["bf16"]
    d = np.abs(p16 - p32)
    flips = np.nonzero(l16 != l32)[0]
    pos = l32.mean()
    m32 = lv.boundary_metrics(l32.tolist(), timestamps, F, T, S)
    m16 = lv.boundary_metrics(l16.tolist(), timestamps, F, T, S)
    print(f"C5: {len(win)} windows, positive share {pos:.3f}; |p16 - p32| median {np.median(d):.2e} max {d.max():.2e}; "
          f"{len(flips)} label flips, max |p32 - 0.5| among them "
          f"{(np.abs(p32[flips] - 0.5).max() if len(flips) else 0):.2e}")
    print("C5 fp32 metrics", {k: m32[k] for k in ("recall", "precision", "f", "f_3", "f_5")})
    print("C5 bf16 metrics", {k: m16[k] for k in ("recall", "precision", "f", "f_3", "f_5")})
    assert 0.2 < pos < 0.8
    assert d.max() <= 5e-2
    if len(flips):
        assert np.abs(p32[flips] - 0.5).max() <= 5 * np.median(d), "labels flipped far from the decision boundary"
    share = len(flips) / len(win)
    for k in ("f", "f_3", "f_5"):
        assert abs(m16[k] - m32[k]) <= max(2 * share, 1e-9) + (0.0 if share == 0 else 0.05), k
    if len(flips) == 0:
        assert m16 == m32
    # the fp32 parity mode against the CPU oracle on 16 windows spread over the video
    pick = np.linspace(0, len(win) - 1, 16).astype(np.int64)
    p = {k: v.detach().cpu() for k, v in models["fp32"].state_dict().items()}
    img = normalize_frames(frames[torch.from_numpy(idx[pick].reshape(-1)).to(DEV)].cpu().numpy().reshape(
        16, T, HW, HW, 3))
    torch.set_num_threads(min(16, len(os.sched_getaffinity(0))))
    with torch.no_grad():
        _, pr, _, _ = om.two_stream(p, img, torch.from_numpy(ids[pick]), torch.from_numpy(mask[pick]),
                                    bn_mode="running")
    e = np.abs(pr[:, 1].numpy() - p32[pick]).max()
    print(f"C5 fp32 native vs oracle on 16 windows: max |dprob| {e:.2e}")
    assert e < 1e-3


def test_c5_batch_stat_bn_vs_oracle():
    """Config 5 under the reference F1 pipeline's BN semantics (test_video_segment_point.py:116-122: running
    statistics dropped, every batch of 16 consecutive windows normalised with its own statistics, batch 16 at :41)
    on the full 1 h video, stride 1 s: fp32 parity mode scored end to end, bf16 vs fp32 labels / F1 on every
    window, and two whole 16-window batches (the batch partition is part of the result) against the CPU oracle in
    its "batch" BN mode within 1e-3."""
    import long_video as lv
    from data.synthetic_dataset import HashTokenizer, normalize_frames
    from oracle import model as om
    from test_video_segment_point import drop_bn_running_stats
    from vcg_hip import ops
    from vcg_hip.build import build_two_stream
    F, T, HW, L, S, BS = 3600, 16, 224, 128, 1, 16
    frames, timestamps, subtitles = lv.synthetic_long_video(F, HW, HW, seed=123, device=DEV)
    win, idx, ids, mask = lv.window_inputs(F, T, S, subtitles, HashTokenizer(), L)
    idx_d, ids_d, mask_d = (torch.from_numpy(a).to(DEV) for a in (idx, ids, mask))
    models = {p: build_two_stream(clip_frame_num=T, seed=123, device=DEV, precision=p, dropout=0.0).eval()
              for p in ("fp32", "bf16")}
    for m in models.values():
        assert drop_bn_running_stats(m) == 53
    with torch.no_grad():  # re-bias the head so that about half the windows are positive (see the test above)
        fr = ops.window_frames_u8(frames, idx_d[:BS].contiguous(), torch.float32, cpad=ops.stem_cpad(torch.float32))
        lg, _ = models["fp32"].forward_staged(fr, ids_d[:BS], mask_d[:BS])
        shift = (lg[:, 0] - lg[:, 1]).median().item()
        for m in models.values():
            m.fusion_head.head.bias.data[1] += shift
            m.native_flat().refresh_shadow(force=True)
    res = {}
    for p, m in models.items():
        sc, lab = lv.score_windows(m, frames, idx_d, ids_d, mask_d, batch_size=BS)
        torch.cuda.synchronize()
        res[p] = (sc.cpu().numpy().astype(np.float64), lab.cpu().numpy())
    p32, l32 = res["fp32"]
    p16, l16 = res["bf16"]
    d = np.abs(p16 - p32)
    flips = np.nonzero(l16 != l32)[0]
    m32 = lv.boundary_metrics(l32.tolist(), timestamps, F, T, S)
    m16 = lv.boundary_metrics(l16.tolist(), timestamps, F, T, S)
    print(f"C5 batch-stat BN: positive share {l32.mean():.3f}; |p16 - p32| median {np.median(d):.2e} max "
          f"{d.max():.2e}; {len(flips)} flips")
    print("C5 batch-stat fp32 metrics", {k: m32[k] for k in ("recall", "precision", "f", "f_3", "f_5")})
    print("C5 batch-stat bf16 metrics", {k: m16[k] for k in ("recall", "precision", "f", "f_3", "f_5")})
    assert 0.05 < l32.mean() < 0.95
    assert d.max() <= 5e-2
    share = len(flips) / len(win)
    for k in ("f", "f_3", "f_5"):
        assert abs(m16[k] - m32[k]) <= max(2 * share, 1e-9) + (0.0 if share == 0 else 0.05), k
    p = {k: v.detach().cpu() for k, v in models["fp32"].state_dict().items()}
    torch.set_num_threads(min(16, len(os.sched_getaffinity(0))))
    for b0 in (0, (len(win) // 2) // BS * BS):
        sel = np.arange(b0, b0 + BS)
        img = normalize_frames(frames[torch.from_numpy(idx[sel].reshape(-1)).to(DEV)].cpu().numpy().reshape(
            BS, T, HW, HW, 3))
        with torch.no_grad():
            _, pr, _, _ = om.two_stream(p, img, torch.from_numpy(ids[sel]), torch.from_numpy(mask[sel]),
                                        bn_mode="batch")
        e = np.abs(pr[:, 1].numpy() - p32[sel]).max()
        print(f"C5 batch-stat fp32 native vs oracle, windows {b0}..{b0 + BS - 1}: max |dprob| {e:.2e}")
        assert e < 1e-3


def test_score_windows_streams_identical():
    """Batch-statistics scoring with the batches spread over 4 HIP streams gives bit-identical scores / labels to
    one stream (each batch is still one forward over exactly its own windows)."""
    import long_video as lv
    from data.synthetic_dataset import HashTokenizer
    from test_video_segment_point import drop_bn_running_stats
    from vcg_hip.build import build_two_stream
    F, T, HW, L = 80, 4, 112, 32
    model = build_two_stream(clip_frame_num=T, seed=123, device=DEV, precision="bf16", dropout=0.0).eval()
    drop_bn_running_stats(model)
    frames, _, subtitles = lv.synthetic_long_video(F, HW, HW, chapter_every=12, seed=8, device=DEV)
    win, idx, ids, mask = lv.window_inputs(F, T, 1, subtitles, HashTokenizer(), L)
    args = [torch.from_numpy(a).to(DEV) for a in (idx, ids, mask)]
    s1, l1 = lv.score_windows(model, frames, *args, batch_size=16, streams=1)
    s4, l4 = lv.score_windows(model, frames, *args, batch_size=16, streams=4)
    torch.cuda.synchronize()
    assert torch.equal(s1, s4) and torch.equal(l1, l4)


def test_c5_stride4_f1_vs_oracle_golden():
    """BASELINE config 5's F1 end to end against the CPU oracle: the reference F1 pipeline's setting
    (test_video_segment_point.py:244-377 -> eval_utils.py:3-92) -- stride 4 s (2 * max_offset,
    flat_video2clip_for_quick_infer.py:66), batch-statistics BN over batches of 16 consecutive windows (:41,116-122),
    fp32 -- over the 1 h synthetic video (896 windows). tests/golden/c5_stride4_batch16.npz holds the oracle's
    prob[:, 1], labels and boundary metrics for every window (tools/oracle/make_golden_c5.py, the oracle run in the
    build container) and the head's logit-1 bias shift it applied; the native fp32 path scores the same windows with
    the same shift. prob within 1e-3; labels equal wherever the oracle's |p - 0.5| exceeds twice the largest
    |dprob| measured (a label may differ only where the probability error can explain it: at random init every
    probability lies within 1e-2 of 0.5, 126 of them within 1e-3); F / F@3 / F@5 (and every recall / precision)
    equal when all labels agree."""
    import long_video as lv
    from data.synthetic_dataset import HashTokenizer
    from test_video_segment_point import drop_bn_running_stats
    from vcg_hip.build import build_two_stream
    g = np.load(os.path.join(GOLD, "c5_stride4_batch16.npz"), allow_pickle=False)
    F, T, HW, L, S, BS = (int(v) for v in g["config"])
    frames, timestamps, subtitles = lv.synthetic_long_video(F, HW, HW, seed=123, device=DEV)
    win, idx, ids, mask = lv.window_inputs(F, T, S, subtitles, HashTokenizer(), L)
    assert np.array_equal(win, g["win"])
    model = build_two_stream(clip_frame_num=T, seed=123, device=DEV, precision="fp32", dropout=0.0).eval()
    assert drop_bn_running_stats(model) == 53
    with torch.no_grad():
        model.fusion_head.head.bias.data[1] += float(g["shift"])
        model.native_flat().refresh_shadow(force=True)
    idx_d, ids_d, mask_d = (torch.from_numpy(a).to(DEV) for a in (idx, ids, mask))
    sc, lab = lv.score_windows(model, frames, idx_d, ids_d, mask_d, batch_size=BS)
    torch.cuda.synchronize()
    p32, l32 = sc.cpu().numpy().astype(np.float64), lab.cpu().numpy()
    ref, ref_lab = g["prob1"], g["labels"]
    d = np.abs(p32 - ref)
    sure = np.abs(ref - 0.5) > 2 * d.max()
    m32 = lv.boundary_metrics(l32.tolist(), timestamps, F, T, S)
    print(f"C5 stride {S} batch-stat fp32 vs oracle: {len(win)} windows, max |dprob| {d.max():.2e}, "
          f"{int((l32 != ref_lab).sum())} label differences ({int((~sure).sum())} windows within 2 max |dprob| of 0.5)")
    print("native", {k: m32[k] for k in ("recall", "precision", "f", "f_3", "f_5")})
    print("oracle", {k: float(g["metric_" + k]) for k in ("recall", "precision", "f", "f_3", "f_5")})
    assert d.max() < 1e-3
    assert np.array_equal(l32[sure], ref_lab[sure])
    if np.array_equal(l32, ref_lab):
        assert m32["gt_cut_points"] == g["gt_cut_points"].tolist()
        assert m32["pred_cut_points"] == g["pred_cut_points"].tolist()
        for k in ("recall", "recall_3", "recall_5", "precision", "precision_3", "precision_5", "f", "f_3", "f_5"):
            assert m32[k] == float(g["metric_" + k]), k


@pytest.mark.parametrize("precision,streams", [("bf16", 3), ("bf16", 1), ("fp32", 3)])
def test_score_windows_groups_identical(precision, streams):
    """Batch-statistics scoring with 4 batches of 16 windows per forward (TwoStream.bn_group: the trunk per batch with
    its own BatchNorm statistics -- the groups' trunks on `streams` HIP streams --, BERT and the head once over all 64
    windows) gives bit-identical scores / labels to one forward per batch (test_video_segment_point.py:41,116-122);
    the final ragged batch included."""
    import long_video as lv
    from data.synthetic_dataset import HashTokenizer
    from test_video_segment_point import drop_bn_running_stats
    from vcg_hip.build import build_two_stream
    F, T, HW, L = 80, 4, 112, 32
    model = build_two_stream(clip_frame_num=T, seed=123, device=DEV, precision=precision, dropout=0.0).eval()
    drop_bn_running_stats(model)
    model.bn_group_streams = streams
    frames, _, subtitles = lv.synthetic_long_video(F, HW, HW, chapter_every=12, seed=8, device=DEV)
    win, idx, ids, mask = lv.window_inputs(F, T, 1, subtitles, HashTokenizer(), L)
    assert len(win) % 16 != 0  # a ragged last batch
    args = [torch.from_numpy(a).to(DEV) for a in (idx, ids, mask)]
    s1, l1 = lv.score_windows(model, frames, *args, batch_size=16)
    s4, l4 = lv.score_windows(model, frames, *args, batch_size=16, groups=4)
    torch.cuda.synchronize()
    assert model.bn_group is None
    assert torch.equal(s1, s4) and torch.equal(l1, l4)
    # and not what one batch of 64 gives (the statistics do span only each group)
    s64, _ = lv.score_windows(model, frames, *args, batch_size=64)
    assert not torch.equal(s1, s64)
