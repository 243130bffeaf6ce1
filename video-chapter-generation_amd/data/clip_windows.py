"""Sliding-window / label / frame-index / subtitle logic of the clip scorer.

Own restatement (vectorised over windows with numpy) of:
  - cut-point parsing      `data/common_utils.py:37-83` (extract_timestamp / extract_first_timestamp)
  - train windows + labels `data/youtube_dataset.py:64-121`
  - eval clip JSON         `video_chapter_youtube_dataset/flat_video2clip_for_quick_infer.py:46-120`
  - frame file index       `youtube_dataset.py:180-190` / `flat_video2clip_for_quick_infer.py:96-106`
  - window subtitles       `youtube_dataset.py:141-151`
  - tokenisation + padding `youtube_dataset.py:156-174`, `infer_youtube_video_dataset.py:284-300`

Everything here is integer / string work on the host and must be bit-exact with the reference:
the IoU test uses the same float64 division and comparison as the reference's Python floats.
"""
import re

import numpy as np

# (pattern, field widths) in the reference's search priority: hh:mm:ss, h:mm:ss, mm:ss, m:ss
_TS_PATTERNS = (re.compile(r"\d{2}:\d{2}:\d{2}"), re.compile(r"\d{1}:\d{2}:\d{2}"),
                re.compile(r"\d{2}:\d{2}"), re.compile(r"\d{1}:\d{2}"))
MAX_OFFSET = 2          # seconds (at 1 fps) a positive window may be off the cut point
TEXT_EXTRA_GAP = 1      # subtitles starting within (s - 1, e + 1) belong to window [s, e)


def extract_timestamp(s):
    """First timestamp of `s` by the reference's pattern priority -> (text, seconds, start, end);
    ("", -1, -1, -1) when there is none. `common_utils.py:37-68`."""
    for pat in _TS_PATTERNS:
        m = pat.search(s)
        if m:
            si, ei = m.span()
            parts = [int(x) for x in s[si:ei].split(":")]
            sec = 0
            for p in parts:
                sec = sec * 60 + p
            return s[si:ei], sec, si, ei
    return "", -1, -1, -1


def extract_first_timestamp(s):
    """Smallest timestamp in `s` and `s` with every timestamp removed. `common_utils.py:71-83`."""
    _, sec, si, ei = extract_timestamp(s)
    best = sec
    desc = s[:si] + s[ei:]
    while sec != -1:
        _, sec, si, ei = extract_timestamp(desc)
        if sec != -1:
            best = min(best, sec)
            desc = desc[:si] + desc[ei:]
    return best, desc


def cut_points_from_timestamps(timestamps, image_num, mode="train", fps=1):
    """Chapter starts (s) kept as ground truth: >= 4 s, and <= image_num (train,
    `youtube_dataset.py:80-87`) or <= image_num - 4 (eval JSON, `flat_video2clip…:52-57`)."""
    hi = image_num if mode == "train" else image_num - 4 * fps
    out = []
    for t in timestamps:
        sec, _ = extract_first_timestamp(t)
        if sec < 4 * fps or sec > hi:
            continue
        out.append(sec)
    return out


def clip_windows(image_num, clip_frame_num, max_offset=MAX_OFFSET):
    """Windows [s, s + T) for s in range(0, N - T, 2 * max_offset) as an int64 [n, 2] array."""
    starts = np.arange(0, image_num - clip_frame_num, 2 * max_offset, dtype=np.int64)
    return np.stack([starts, starts + clip_frame_num], axis=1)


def clip_labels(windows, cut_points, clip_frame_num, max_offset=MAX_OFFSET):
    """1 where IoU([s, e), [cp - T/2, cp + T/2)) >= (T - off) / (T + off) for some cut point."""
    windows = np.asarray(windows, dtype=np.int64).reshape(-1, 2)
    if len(cut_points) == 0 or len(windows) == 0:
        return np.zeros(len(windows), dtype=np.int64)
    half = clip_frame_num // 2
    s = windows[:, :1]
    e = windows[:, 1:]
    cp = np.asarray(cut_points, dtype=np.int64)[None, :]
    ps, pe = cp - half, cp + half
    inter = np.minimum(e, pe) - np.maximum(s, ps)
    union = np.maximum(e, pe) - np.minimum(s, ps)
    iou = inter.astype(np.float64) / union.astype(np.float64)
    thr = (clip_frame_num - max_offset) / (clip_frame_num + max_offset)
    return (iou >= thr).any(axis=1).astype(np.int64)


def frame_numbers(start, clip_frame_num, image_num):
    """1-based frame file numbers (`%05d.jpg`) of window [start, start + T): +1 near either end of
    the video, +3 elsewhere (the reference's ffmpeg alignment fix)."""
    off = 1 if (start <= 2 or start >= image_num - clip_frame_num - 2) else 3
    return np.arange(start, start + clip_frame_num, dtype=np.int64) + off


def frame_index_table(windows, image_num):
    """0-based frame indices [n_windows, T] for every window (the GPU gather's index map)."""
    windows = np.asarray(windows, dtype=np.int64).reshape(-1, 2)
    T = int(windows[0, 1] - windows[0, 0]) if len(windows) else 0
    s = windows[:, :1]
    edge = (s <= 2) | (s >= image_num - T - 2)
    return s + np.arange(T, dtype=np.int64)[None, :] + np.where(edge, 0, 2)


def window_text(subtitles, start, end, gap=TEXT_EXTRA_GAP, fps=1):
    """Subtitle texts with start - gap < sub.start < end + gap, each appended after a single space
    unless the text so far is empty (so an empty first subtitle adds no separator)."""
    out = ""
    for sub in subtitles:
        if start - gap * fps < sub["start"] * fps < end + gap * fps:
            out = out + " " + sub["text"] if out else out + sub["text"]
    return out


def encode_text(tokenizer, text, max_text_len):
    """"[CLS] " + text -> tokens truncated to L, "[PAD]"-padded; mask 1/0 (no [SEP])."""
    tokens = tokenizer.tokenize("[CLS] " + text)[:max_text_len]
    n = len(tokens)
    tokens = tokens + ["[PAD]"] * (max_text_len - n)
    ids = np.asarray(tokenizer.convert_tokens_to_ids(tokens), dtype=np.int64)
    mask = np.zeros(max_text_len, dtype=np.int64)
    mask[:n] = 1
    return ids, mask


def video_clip_infos(vid, image_dir, image_num, timestamps, subtitles, clip_frame_num, fps=1):
    """The eval clip-JSON records of one video (`flat_video2clip_for_quick_infer.py:62-118`):
    image_paths, text_clip, clip_label, clip_start_end, cut_points, vid."""
    import os

    cut_points = cut_points_from_timestamps(timestamps, image_num, mode="eval", fps=fps)
    max_offset = 2 * fps
    win = clip_windows(image_num, clip_frame_num, max_offset)
    labels = clip_labels(win, cut_points, clip_frame_num, max_offset)
    out = []
    for (s, e), lab in zip(win.tolist(), labels.tolist()):
        out.append({
            "image_paths": [os.path.join(image_dir, vid, "%05d.jpg" % k)
                            for k in frame_numbers(s, clip_frame_num, image_num).tolist()],
            "text_clip": window_text(subtitles, s, e, TEXT_EXTRA_GAP, fps),
            "clip_label": int(lab),
            "clip_start_end": [int(s), int(e)],
            "cut_points": list(cut_points),
            "vid": vid,
        })
    return out


def window_clip_indices(target_idx, n_clips, clip_frame_num, window_size, max_offset=MAX_OFFSET):
    """Clip indices of the window around `target_idx` (youtube_dataset.py:438-446, WindowClipDataset): 2w+1 clips
    `skip = T // (2 * max_offset)` apart (so consecutive window clips do not overlap), -1 where the window runs off
    either end of the video (the reference pads those clips with zero frames / text / mask)."""
    skip = clip_frame_num // (2 * max_offset)
    return [i if 0 <= i < n_clips else -1
            for i in range(target_idx - skip * window_size, target_idx + skip * window_size + 1, skip)]


def window_clip_info(windows, target_idx, clip_frame_num, window_size, image_num, max_offset=MAX_OFFSET):
    """The reference's `clips_info` dict (youtube_dataset.py:507-527) as int64 arrays: clip_start_frame [2w+1]
    (-1 for padding clips), total_frames, target_clip_idx, total_num_clips."""
    windows = np.asarray(windows, dtype=np.int64).reshape(-1, 2)
    idx = window_clip_indices(target_idx, len(windows), clip_frame_num, window_size, max_offset)
    starts = np.array([windows[i, 0] if i >= 0 else -1 for i in idx], dtype=np.int64)
    return {"clip_start_frame": starts, "total_frames": np.int64(image_num), "target_clip_idx": np.int64(target_idx),
            "total_num_clips": np.int64(len(windows))}
