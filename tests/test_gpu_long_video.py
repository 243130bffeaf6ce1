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
