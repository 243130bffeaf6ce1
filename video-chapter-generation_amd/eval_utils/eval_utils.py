"""Clip-label -> cut-point conversion and cut-point recall / precision (drop-in for reference
eval_utils/eval_utils.py:3-92).

Semantics kept from the reference:
* windows i are `clip_frame_num` seconds long and start every `2*max_offset` seconds;
* a run of positive windows [i0, i1) becomes the cut point round((begin + end - 1) / 2) with
  begin = i0*2*max_offset and end = (i1-1)*2*max_offset + clip_frame_num, using Python's round
  (half to even);
* a run still open at the end of the list is dropped (no closing 0 was seen);
* recall / precision count a hit at exact, +-3 s and +-5 s; precision values are None when there
  are no predicted cut points.
"""


def convert_clip_label2cut_point(clip_label_array, clip_frame_num, max_offset):
    stride = 2 * max_offset
    cut_points = []
    run_start = None
    for i, lab in enumerate(clip_label_array):
        if lab == 1 and run_start is None:
            run_start = i
        elif lab == 0 and run_start is not None:
            begin = run_start * stride
            end = (i - 1) * stride + clip_frame_num
            cut_points.append(round((begin + end - 1) / 2))
            run_start = None
    return cut_points


def _hit_rates(queries, targets):
    """Fractions of `queries` that have a target at distance 0, <=3, <=5."""
    n = len(queries)
    exact = sum(1 for q in queries if any(q == t for t in targets))
    within3 = sum(1 for q in queries if any(abs(q - t) <= 3 for t in targets))
    within5 = sum(1 for q in queries if any(abs(q - t) <= 5 for t in targets))
    return exact / n, within3 / n, within5 / n


def calculate_pr(gt_cut_points, pred_cut_points):
    """-> (recall, recall@3s, recall@5s, precision, precision@3s, precision@5s)."""
    recall, recall_3, recall_5 = _hit_rates(gt_cut_points, pred_cut_points)
    precision = precision_3 = precision_5 = None
    if len(pred_cut_points) > 0:
        precision, precision_3, precision_5 = _hit_rates(pred_cut_points, gt_cut_points)
    return recall, recall_3, recall_5, precision, precision_3, precision_5
