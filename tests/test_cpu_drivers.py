"""CPU tests of the driver-side host logic: LR schedule, per-video metric pipelines (with the
reference's quirks), synthetic datasets (sample tuples through the real window logic)."""
import math
import os
import random

import numpy as np
import pytest
import torch

from train_video_segment_point import TrainerConfig, lr_multiplier
from eval_utils.video_metrics import evaluate_videos, trainer_video_auc_map
from eval_utils.eval_utils import calculate_pr, convert_clip_label2cut_point


def test_lr_schedule_matches_reference_formula():
    c = TrainerConfig(warmup_epochs=3, final_epochs=270, lr_decay_type="cosine")
    assert lr_multiplier(c, 0) == 1e-2                     # max(0/3, 0.01)
    assert lr_multiplier(c, 1) == pytest.approx(1 / 3)
    assert lr_multiplier(c, 3) == pytest.approx(0.5 * (1 + math.cos(math.pi * 3 / 270)))
    assert lr_multiplier(c, 270) == 0.001                  # progress 1 -> 0 -> floor
    assert lr_multiplier(c, 500) == 0.001
    e = TrainerConfig(warmup_epochs=0, final_epochs=100, lr_decay_type="exp")
    assert [lr_multiplier(e, x) for x in (10, 30, 50, 20, 90)] == [1, 0.1, 0.01, 0.001, 0.001]
    with pytest.raises(RuntimeError):
        lr_multiplier(TrainerConfig(warmup_epochs=0, final_epochs=10, lr_decay_type="step"), 5)
    # the reference driver's defaults: warmup = epochs // 100 = 0 at 50 epochs -> straight to cosine
    d = TrainerConfig(warmup_epochs=0, final_epochs=0)
    assert lr_multiplier(d, 1) == 0.001


def _infos(vids_labels_scores):
    out = []
    for vid, labels, scores in vids_labels_scores:
        for k, (l, s) in enumerate(zip(labels, scores)):
            out.append({"vid": vid, "clip_label": l, "pred_score": s, "pred_label": int(s > 0.5),
                        "clip_start_end": [4 * k, 4 * k + 16], "cut_points": [20]})
    return out


def test_trainer_metric_drops_last_video():
    a = ("a", [0, 1, 0, 1], [0.1, 0.9, 0.2, 0.8])        # perfect ranking: AUC 1
    b = ("b", [0, 1, 1, 0], [0.9, 0.1, 0.2, 0.8])        # inverted: AUC 0 — never scored (last video)
    auc, ap = trainer_video_auc_map(_infos([a, b]))
    assert auc == 1.0 and ap == 1.0
    auc, ap = trainer_video_auc_map(_infos([b, a]))
    assert auc == 0.0


def test_evaluate_videos_double_counts_first_clip_and_adds_last():
    from sklearn import metrics
    a = ("a", [1, 0, 0, 1], [0.9, 0.2, 0.6, 0.7])
    infos = _infos([a])
    res, vid2cut = evaluate_videos(infos, 16, 2, random.Random(0))
    labels = [1] + a[1]                                   # first clip appears twice
    scores = [0.9] + a[2]
    fpr, tpr, _ = metrics.roc_curve(labels, scores, pos_label=1)
    assert res["auc"] == pytest.approx(metrics.auc(fpr, tpr))
    assert res["mAP"] == pytest.approx(metrics.average_precision_score(labels, scores))
    preds = [1] + [int(s > 0.5) for s in a[2]]
    assert vid2cut["a"]["second_gt_cut_points"] == convert_clip_label2cut_point(labels, 16, 2)
    assert vid2cut["a"]["second_pred_cut_points"] == convert_clip_label2cut_point(preds, 16, 2)
    r = calculate_pr(vid2cut["a"]["second_gt_cut_points"], vid2cut["a"]["second_pred_cut_points"])
    assert res["recall"] == pytest.approx(r[0])


def test_synthetic_datasets_produce_reference_tuples():
    from data.synthetic_dataset import HashTokenizer, InferYoutubeClipDataset, SyntheticVideoCorpus, YoutubeClipDataset
    from data import clip_windows as cw
    corpus = SyntheticVideoCorpus(3, min_len=40, max_len=60, H=16, W=16, seed=5)
    tok = HashTokenizer()
    random.seed(0)
    ds = YoutubeClipDataset(corpus, tok, 8, 24)
    img, ids, mask, label = ds[1]
    assert img.shape == (8, 3, 16, 16) and img.dtype == torch.float32
    assert ids.shape == (24,) and ids[0] == 101 and mask.dtype == torch.int64 and label in (0, 1)
    assert torch.equal(ids * (1 - mask), torch.zeros_like(ids))   # pad id 0 where mask 0
    inf = InferYoutubeClipDataset(corpus, tok, 8, 24)
    n = sum(len(cw.clip_windows(corpus.image_num[v], 8)) for v in corpus.vids)
    assert len(inf) == n
    img, ids, mask, label = inf[3]
    info = inf.all_clip_infos[3]
    s = info["clip_start_end"][0]
    frames = corpus.frames(info["vid"], cw.frame_numbers(s, 8, corpus.image_num[info["vid"]]) - 1)
    mean = torch.tensor([0.485, 0.456, 0.406])
    std = torch.tensor([0.229, 0.224, 0.225])
    ref = ((torch.from_numpy(frames).float() / 255.0 - mean) / std).permute(0, 3, 1, 2)
    assert torch.equal(img, ref)
    assert label == info["clip_label"]
    # deterministic frames (rebuilt anywhere from the seed)
    assert np.array_equal(corpus.frames("synvid0000", [3]), SyntheticVideoCorpus(3, 40, 60, H=16, W=16, seed=5).frames("synvid0000", [3]))


@pytest.mark.parametrize("ckpt", ["ck/", "ck/run", "ck/run.pth"])
def test_ddp_checkpoint_search_matches_save_names(tmp_path, ckpt):
    """find_latest_checkpoint: a directory ("DIR/") is searched as the reference does (every DIR/*.pth matched by
    `_(\\d+)(?:_score_[\\d.]+)?\\.pth$`, whatever its prefix: other_9.pth wins); a name prefix ("DIR/run", "DIR/run.pth"),
    where the reference finds nothing, is searched where checkpoint_path writes (other prefixes ignored). Names that
    do not end in .pth are ignored either way."""
    import train_video_segment_ddp as drv
    path = str(tmp_path / ckpt)
    os.makedirs(tmp_path / "ck", exist_ok=True)
    for ep, best in ((1, None), (3, 0.25), (2, None)):
        p = drv.checkpoint_path(path, ep, best or 0.0, best is not None)
        open(p, "w").close()
    open(tmp_path / "ck" / "other_9.pth", "w").close()
    open(tmp_path / "ck" / "run_11.pth.tmp", "w").close()
    found, ep = drv.find_latest_checkpoint(path)
    if ckpt.endswith("/"):
        assert ep == 9 and found == str(tmp_path / "ck" / "other_9.pth")
        assert drv.find_latest_checkpoint(str(tmp_path / "ck"))[1] == 9  # (an existing directory without the "/")
    else:
        assert ep == 3 and found == drv.checkpoint_path(path, 3, 0.25, True)
    assert drv.find_latest_checkpoint(str(tmp_path / "none" / "x"))[0] is None


@pytest.mark.parametrize("extra", [False, True])
def test_ddp_fit_checkpoint_cadence(tmp_path, extra):
    """The reference's cadence (train_video_segment_ddp.py:271-290): validation epochs write a best checkpoint when
    the metric improves and never a regular one (`elif`); other epochs write a regular one every save_every epochs.
    save_on_val_epochs adds the regular save on validation epochs without a new best."""
    import train_video_segment_ddp as drv
    tr = drv.DDPTrainer.__new__(drv.DDPTrainer)
    results = iter([0.5, 0.4, float("nan")])  # epochs 2, 4, 6: best, worse, NaN
    saved = []
    tr.config = type("C", (), {"max_epochs": 7})()
    tr.start_epoch, tr.best_result, tr.rank, tr.test_dataset = 0, float("-inf"), 1, object()
    tr.run_epoch = lambda split, epoch: next(results) if split == "infer_test" else None
    tr.save_checkpoint = lambda epoch, best, is_best=False: saved.append((epoch, is_best))
    tr.fit(val_every=2, save_every=3, save_on_val_epochs=extra)
    want = [(2, True), (3, False)] + ([(6, False)] if extra else [])
    assert saved == want and tr.best_result == 0.5
