"""CPU tests of the window / label / frame-index / subtitle logic and the
clip-JSON format: data/clip_windows.py (product, vectorised) against oracle/windows.py (plain-loop
restatement) and tests/golden/windows.json (reference extract_first_timestamp outputs + known
answers). Everything here is integer/string work: equality is exact."""
import json
import os
import random

import numpy as np
import pytest

from data import clip_windows as cw
from oracle import windows as ow

GOLD = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "windows.json")))


def test_extract_first_timestamp_matches_reference():
    for case in GOLD["extract_first_timestamp"]:
        sec, desc = cw.extract_first_timestamp(case["s"])
        assert (sec, desc) == (case["sec"], case["desc"]), case["s"]


def test_known_answers_video40():
    k = GOLD["known"]["video40"]
    win = cw.clip_windows(k["image_num"], k["T"])
    assert win.tolist() == k["windows"] == ow.clip_windows(k["image_num"], k["T"])
    lab = cw.clip_labels(win, k["cut_points"], k["T"])
    assert lab.tolist() == k["labels"]
    assert [ow.clip_label(s, e, k["cut_points"], k["T"]) for s, e in k["windows"]] == k["labels"]
    for s, key in ((0, "frames_s0"), (4, "frames_s4"), (20, "frames_s20")):
        assert cw.frame_numbers(s, k["T"], k["image_num"]).tolist() == k[key]
        assert ow.frame_numbers(s, s + k["T"], k["image_num"], k["T"]) == k[key]


def test_known_answers_subtitles_and_filters():
    sub = GOLD["known"]["subtitles"]
    s, e = sub["window"]
    assert cw.window_text(sub["subs"], s, e) == sub["text"] == ow.window_text(sub["subs"], s, e)
    f = GOLD["known"]["filters"]
    for mode in ("train", "eval"):
        ts = [f"{x // 60}:{x % 60:02d} chapter" if x >= 0 else "no time" for x in f["secs"]]
        assert cw.cut_points_from_timestamps(ts, f["image_num"], mode=mode) == f[mode]
        assert ow.cut_points(f["secs"], f["image_num"], mode) == f[mode]


@pytest.mark.parametrize("T", [4, 8, 16, 20])
def test_vectorised_windows_match_loop_restatement(T):
    rng = random.Random(1234 + T)
    for _ in range(200):
        n = rng.randint(T + 1, 900)
        cps = sorted(rng.sample(range(-5, n + 10), k=rng.randint(0, 12)))
        win = cw.clip_windows(n, T)
        assert win.tolist() == ow.clip_windows(n, T)
        lab = cw.clip_labels(win, cps, T).tolist()
        assert lab == [ow.clip_label(s, e, cps, T) for s, e in win.tolist()]
        table = cw.frame_index_table(win, n)
        for (s, e), row in zip(win.tolist(), table.tolist()):
            nums = ow.frame_numbers(s, e, n, T)
            assert cw.frame_numbers(s, T, n).tolist() == nums
            assert row == [x - 1 for x in nums]  # 0-based gather index = file number - 1


def test_window_text_matches_loop_restatement():
    rng = random.Random(7)
    for _ in range(300):
        subs = [{"start": round(rng.uniform(0, 120), 2), "text": rng.choice(["", "hi", "a b", "x"])}
                for _ in range(rng.randint(0, 30))]
        s = rng.randint(0, 100)
        assert cw.window_text(subs, s, s + 16) == ow.window_text(subs, s, s + 16)


def test_edge_cases_empty_and_short():
    assert cw.clip_windows(16, 16).shape == (0, 2)          # N == T: range(0, 0) is empty
    assert cw.clip_windows(17, 16).tolist() == [[0, 16]]
    assert cw.clip_labels(np.zeros((0, 2), np.int64), [5], 16).shape == (0,)
    assert cw.clip_labels(cw.clip_windows(40, 16), [], 16).tolist() == [0] * 6
    assert cw.extract_first_timestamp("") == (-1, "")


class _Tok:
    """Whitespace tokenizer with a fixed vocabulary (the real one is bert-base-uncased, not shipped)."""
    vocab = {"[PAD]": 0, "[CLS]": 101, "[UNK]": 100}

    def tokenize(self, s):
        return s.split()

    def convert_tokens_to_ids(self, toks):
        return [self.vocab.setdefault(t, 1000 + len(self.vocab)) for t in toks]


def test_encode_text_pads_truncates_and_masks():
    tok = _Tok()
    ids, mask = cw.encode_text(tok, "hello world", 6)
    assert ids.tolist()[0] == 101 and ids.tolist()[3:] == [0, 0, 0]
    assert mask.tolist() == [1, 1, 1, 0, 0, 0]
    ids, mask = cw.encode_text(tok, " ".join(["w"] * 20), 6)
    assert mask.tolist() == [1] * 6 and len(ids) == 6


def test_clip_json_records(tmp_path):
    subs = [{"start": 5.0, "text": "intro"}, {"start": 30.0, "text": "second part"}]
    recs = cw.video_clip_infos("vid0", "/frames", 60, ["0:00 a", "0:20 b", "0:58 too late"], subs, 16)
    assert [r["clip_start_end"] for r in recs] == ow.clip_windows(60, 16)
    assert all(r["cut_points"] == [20] for r in recs)          # 58 > 60 - 4 dropped, 0 < 4 dropped
    assert [r["clip_label"] for r in recs] == [ow.clip_label(s, e, [20], 16) for s, e in ow.clip_windows(60, 16)]
    r = recs[2]  # s = 8
    assert r["image_paths"][0] == "/frames/vid0/%05d.jpg" % (8 + 3)
    assert r["text_clip"] == ow.window_text(subs, 8, 24)
    p = tmp_path / "clips.json"
    p.write_text(json.dumps(recs))
    assert json.loads(p.read_text()) == recs


def test_long_video_host_side_and_metrics():
    """long_video.py host logic: stride-1 windows, the reference frame-index rule, text encoding, and the
    cut-point metrics at a window step of 1 s (eval_utils with max_offset = stride / 2)."""
    import long_video as lv
    from data import clip_windows as cw
    from data.synthetic_dataset import HashTokenizer
    subs = [{"start": 1.0, "text": "a b"}, {"start": 9.5, "text": "c"}]
    win, idx, ids, mask = lv.window_inputs(30, 8, 1, subs, HashTokenizer(), 16)
    assert win.shape == (22, 2) and np.array_equal(win[:, 0], np.arange(22))
    assert np.array_equal(idx, cw.frame_index_table(win, 30))
    assert ids[0, 0] == 101 and mask[0].sum() == 3  # "[CLS] a b"
    # labels 1 for windows 3..5 (stride 1, T = 8): begin 3, end 5 + 8 -> round((3 + 13 - 1) / 2) = round(7.5) = 8
    labels = [0, 0, 0, 1, 1, 1, 0] + [0] * 15
    m = lv.boundary_metrics(labels, ["0:00 intro", "0:08 two", "0:29 late"], 30, 8, 1)
    assert m["gt_cut_points"] == [8] and m["pred_cut_points"] == [8]
    assert m["recall"] == 1.0 and m["precision"] == 1.0 and m["f"] == 1.0


def test_window_clip_indices_known_answers():
    """WindowClipDataset's window around a target clip (youtube_dataset.py:438-446): with T = 16 and max_offset = 2
    clips start every 4 s and window clips are skip = 4 clip indices (16 s) apart; off-video clips are -1."""
    from data.clip_windows import clip_windows, window_clip_indices, window_clip_info
    assert window_clip_indices(10, 30, 16, 2) == [2, 6, 10, 14, 18]
    assert window_clip_indices(1, 30, 16, 2) == [-1, -1, 1, 5, 9]
    assert window_clip_indices(28, 30, 16, 1) == [24, 28, -1]
    assert window_clip_indices(0, 1, 16, 0) == [0]
    assert window_clip_indices(5, 30, 8, 1) == [3, 5, 7]  # T = 8: skip 2
    w = clip_windows(120, 16)  # 26 clips
    info = window_clip_info(w, 3, 16, 1, 120)
    assert info["clip_start_frame"].tolist() == [-1, 12, 28]
    assert int(info["total_num_clips"]) == len(w) == 26 and int(info["target_clip_idx"]) == 3
