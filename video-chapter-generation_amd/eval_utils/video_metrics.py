"""Per-video evaluation of clip scores: the metric pipelines of the two drivers, as functions.

- `trainer_video_auc_map` restates the validation block of `Trainer.run_epoch`
  (`train_video_segment_point.py:257-279`). It keeps the reference's quirk: a video's AUC/AP is
  computed only when the NEXT video starts, so the last video is never scored.
- `evaluate_videos` restates the test driver (`test_video_segment_point.py:244-377`): per-video AUC/AP,
  cut points from the clip labels (`convert_clip_label2cut_point`), and recall / precision / F at 0, ±3
  and ±5 s (`calculate_pr`), for the model and for a seeded random baseline. It also keeps the reference's
  double-counted first clip of every video (it is appended at re-init and again right after) and its
  explicit "add last vid" step.
"""
import random as _random

from sklearn import metrics

from .eval_utils import calculate_pr, convert_clip_label2cut_point


def _auc_ap(labels, scores):
    fpr, tpr, _ = metrics.roc_curve(labels, scores, pos_label=1)
    return metrics.auc(fpr, tpr), metrics.average_precision_score(labels, scores)


def trainer_video_auc_map(all_clip_infos):
    """(mean AUC, mean AP) over all videos but the last, in clip order."""
    aucs, aps = [], []
    vid, scores, labels = "", [], []
    for info in all_clip_infos:
        if vid != info["vid"]:
            vid = info["vid"]
            if labels:
                a, p = _auc_ap(labels, scores)
                aucs.append(a)
                aps.append(p)
            scores, labels = [], []
        scores.append(info["pred_score"])
        labels.append(info["clip_label"])
    mean = lambda xs: float(sum(xs) / len(xs)) if xs else float("nan")  # noqa: E731
    return mean(aucs), mean(aps)


class _Acc:
    def __init__(self):
        self.r, self.r3, self.r5, self.p, self.p3, self.p5 = ([] for _ in range(6))

    def add(self, res):
        recall, recall_3, recall_5, precision, precision_3, precision_5 = res
        if recall is not None:
            self.r.append(recall); self.r3.append(recall_3); self.r5.append(recall_5)  # noqa: E702
        if precision is not None:
            self.p.append(precision); self.p3.append(precision_3); self.p5.append(precision_5)  # noqa: E702

    def summary(self):
        # the reference divides unguarded (ZeroDivisionError on an empty list or P = R = 0); nan here
        avg = lambda xs: sum(xs) / len(xs) if xs else float("nan")  # noqa: E731
        r, r3, r5, p, p3, p5 = (avg(x) for x in (self.r, self.r3, self.r5, self.p, self.p3, self.p5))
        f = lambda a, b: 2 * a * b / (a + b) if (a + b) else float("nan")  # noqa: E731
        return {"recall": r, "recall@3": r3, "recall@5": r5, "precision": p, "precision@3": p3,
                "precision@5": p5, "f-score": f(r, p), "f-score@3": f(r3, p3), "f-score@5": f(r5, p5)}


def evaluate_videos(all_clip_infos, clip_frame_num, max_offset=2, rng=None):
    """Test-driver metrics. Each record needs vid, clip_label, pred_score, pred_label,
    clip_start_end and cut_points. Returns (results dict, vid2cut_points)."""
    rng = rng or _random.Random(123)
    aucs, maps = [], []
    model_acc, rand_acc = _Acc(), _Acc()
    vid2cut = {}

    def close_video(vid, gt, scores, preds, duration, gt_cut_points):
        a, p = _auc_ap(gt, scores)
        aucs.append(a)
        maps.append(p)
        gt_cp = convert_clip_label2cut_point(gt, clip_frame_num, max_offset)
        pred_cp = convert_clip_label2cut_point(preds, clip_frame_num, max_offset)
        rand_cp = [rng.randint(0, duration - 1) for _ in range(len(gt_cut_points))]
        vid2cut[vid] = {"second_gt_cut_points": gt_cp, "second_pred_cut_points": pred_cp}
        model_acc.add(calculate_pr(gt_cp, pred_cp))
        rand_acc.add(calculate_pr(gt_cp, rand_cp))

    vid, gt, scores, preds, duration, cps = "", [], [], [], 0, []
    for info in all_clip_infos:
        if vid != info["vid"]:
            if gt:
                close_video(vid, gt, scores, preds, duration, cps)
            vid = info["vid"]
            gt, scores, preds = [info["clip_label"]], [info["pred_score"]], [info["pred_label"]]
        gt.append(info["clip_label"])
        scores.append(info["pred_score"])
        preds.append(info["pred_label"])
        duration = info["clip_start_end"][1]
        cps = info["cut_points"]
    close_video(vid, gt, scores, preds, duration, cps)  # "add last vid"

    res = {"mAP": sum(maps) / len(maps), "auc": sum(aucs) / len(aucs)}
    res.update(model_acc.summary())
    res.update({k + "_rand": v for k, v in rand_acc.summary().items()})
    return res, vid2cut
