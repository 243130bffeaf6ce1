"""TEST INFRASTRUCTURE ONLY — plain-loop restatement of the reference's window / label / frame-index
/ subtitle logic, the checker for `data/clip_windows.py`.

The reference modules that hold this logic cannot be imported in this image:
`data/youtube_dataset.py` needs torchvision and `flat_video2clip_for_quick_infer.py` needs
`youtube_transcript_api` (via `dataset_process_scripts.load_dataset_utils`). So this file restates
the loops statement by statement. Its pins are the known answers in `tests/golden/windows.json`,
which are hand-derived from the reference lines cited below, and the reference's own
`data/common_utils.extract_first_timestamp`, which is importable here; see
`tools/oracle/make_golden_data.py`.
"""


def clip_windows(image_num, clip_frame_num, max_offset=2):
    # youtube_dataset.py:91 / flat_video2clip_for_quick_infer.py:66
    return [[s, s + clip_frame_num] for s in range(0, image_num - clip_frame_num, 2 * max_offset)]


def clip_label(start_t, end_t, cut_points, clip_frame_num, max_offset=2):
    # youtube_dataset.py:99-114 (break on first hit) == flat_video2clip…:73-84 (no break)
    half = int(clip_frame_num // 2)
    label = 0
    for cp in cut_points:
        cs, ce = cp - half, cp + half
        a = max(start_t, cs)
        mi = min(start_t, cs)
        b = min(end_t, ce)
        ma = max(end_t, ce)
        iou = (b - a) / (ma - mi)
        if iou >= (clip_frame_num - max_offset) / (clip_frame_num + max_offset):
            label = 1
            break
    return label


def frame_numbers(clip_start_sec, clip_end_sec, image_num, clip_frame_num):
    # youtube_dataset.py:180-190 / flat_video2clip…:96-106 ("%05d.jpg" numbers)
    out = []
    for idx in range(clip_start_sec, clip_end_sec):
        if clip_start_sec <= 2 or clip_start_sec >= image_num - clip_frame_num - 2:
            out.append(idx + 1)
        else:
            out.append(idx + 3)
    return out


def window_text(subtitles, clip_start_sec, clip_end_sec, gap=1):
    # youtube_dataset.py:141-151
    text_clip = ""
    for sub in subtitles:
        text = sub["text"]
        start_sec = sub["start"]
        if clip_start_sec - gap < start_sec < clip_end_sec + gap:
            if len(text_clip) == 0:
                text_clip += text
            else:
                text_clip += " " + text
    return text_clip


def cut_points(first_timestamps_sec, image_num, mode):
    # train: youtube_dataset.py:78-87 (sec < 4 or sec > image_num dropped);
    # eval:  flat_video2clip…:50-57 (sec < 4 or sec > image_num - 4 dropped)
    out = []
    for sec in first_timestamps_sec:
        if sec < 4:
            continue
        if mode == "train" and sec > image_num:
            continue
        if mode != "train" and sec > image_num - 4:
            continue
        out.append(sec)
    return out


def youtube_clip_item(img_dir, vid, timestamps_sec, subtitles, tokenizer, clip_frame_num, max_text_len, rng):
    """YoutubeClipDataset.__getitem__ (youtube_dataset.py:64-194) for one video, statement by statement, with
    `rng` in place of the module-level `random` and ToTensor + Normalize written out (PIL decode, /255, (x -
    mean) / std in fp32). Returns (img_clip f32 [T,3,H,W] as nested lists -> numpy by the caller, ids, mask,
    label, (clip_start_sec, clip_end_sec))."""
    import glob
    import os

    import numpy as np
    from PIL import Image

    image_path = os.path.join(img_dir, vid)
    image_num = len(glob.glob(image_path + "/*.jpg"))
    cps = []
    for sec in timestamps_sec:  # :73-87
        if sec < 4:
            continue
        if sec > image_num:
            continue
        cps.append(sec)
    max_offset = 2
    clips = [[s, s + clip_frame_num] for s in range(0, image_num - clip_frame_num, 2 * max_offset)]
    pos, neg = [], []
    for idx, (s, e) in enumerate(clips):  # :96-117
        if clip_label(s, e, cps, clip_frame_num, max_offset):
            pos.append(idx)
        else:
            neg.append(idx)
    is_positive = 0 if not pos else rng.sample([0, 1], k=1)[0]  # :121-125
    clip = clips[rng.sample(pos, k=1)[0]] if is_positive else clips[rng.sample(neg, k=1)[0]]
    s, e = clip
    text_clip = "[CLS] " + window_text(subtitles, s, e)  # :141-154
    tokens = tokenizer.tokenize(text_clip)[:max_text_len]  # :155-166
    attention_mask = [1] * len(tokens)
    if len(tokens) < max_text_len:
        attention_mask += [0] * (max_text_len - len(tokens))
        tokens += ["[PAD]"] * (max_text_len - len(tokens))
    ids = tokenizer.convert_tokens_to_ids(tokens)
    mean = np.array([0.485, 0.456, 0.406], dtype=np.float32)
    std = np.array([0.229, 0.224, 0.225], dtype=np.float32)
    imgs = []
    for n in frame_numbers(s, e, image_num, clip_frame_num):  # :176-192
        with Image.open(os.path.join(image_path, "%05d.jpg" % n)) as im:
            a = np.asarray(im.convert("RGB"), dtype=np.float32) / np.float32(255.0)
        imgs.append(((a - mean) / std).transpose(2, 0, 1))
    return np.stack(imgs), ids, attention_mask, 1 if is_positive else 0, (s, e)


def window_clip_item(img_dir, vid, timestamps_sec, subtitles, tokenizer, clip_frame_num, max_text_len, window_size,
                     rng):
    """WindowClipDataset.__getitem__ (youtube_dataset.py:389-536) statement by statement, `rng` for the module-level
    `random`, ToTensor + Normalize written out. Returns (img_clips [2w+1, T, 3, H, W] numpy (zeros for padding
    clips), ids [2w+1][L], masks [2w+1][L], label, clip_start_frames, image_num, target_idx, n_clips)."""
    import glob
    import os

    import numpy as np
    from PIL import Image

    fps = 1
    image_path = os.path.join(img_dir, vid)
    image_num = len(glob.glob(image_path + "/*.jpg"))
    cps = [sec for sec in timestamps_sec if not (sec < 4 * fps or sec > image_num - 4 * fps)]  # :398-403
    max_offset = 2 * fps
    clips = [[s, s + clip_frame_num] for s in range(0, image_num - clip_frame_num, 2 * max_offset)]
    pos, neg = [], []
    for idx, (s, e) in enumerate(clips):
        (pos if clip_label(s, e, cps, clip_frame_num, max_offset) else neg).append(idx)
    is_positive = rng.choice([0, 1]) if pos else 0  # :428
    target_idx = rng.choice(pos if is_positive else neg)
    window_indices = []
    skip = clip_frame_num // (2 * max_offset)  # :432-438
    for idx in range(target_idx - skip * window_size, target_idx + skip * window_size + 1, skip):
        window_indices.append(idx if 0 <= idx < len(clips) else -1)
    mean = np.array([0.485, 0.456, 0.406], dtype=np.float32)
    std = np.array([0.229, 0.224, 0.225], dtype=np.float32)
    imgs, ids, masks, shape = [], [], [], None
    for idx in window_indices:
        if idx == -1:
            imgs.append(None)
            ids.append([0] * max_text_len)
            masks.append([0] * max_text_len)
            continue
        s, e = clips[idx]
        frames = []
        for n in frame_numbers(s, e, image_num, clip_frame_num):
            with Image.open(os.path.join(image_path, "%05d.jpg" % n)) as im:
                a = np.asarray(im.convert("RGB"), dtype=np.float32) / np.float32(255.0)
            frames.append(((a - mean) / std).transpose(2, 0, 1))
        imgs.append(np.stack(frames))
        shape = imgs[-1].shape
        text_clip = "[CLS] "  # :479-483
        for sub in subtitles:
            if s - fps < sub["start"] < e + fps:
                text_clip += sub["text"] + " "
        tokens = tokenizer.tokenize(text_clip)[:max_text_len]
        mask = [1] * len(tokens)
        pad = max_text_len - len(tokens)
        if pad > 0:
            tokens.extend(["[PAD]"] * pad)
            mask.extend([0] * pad)
        ids.append(tokenizer.convert_tokens_to_ids(tokens))
        masks.append(mask)
    img_clips = np.stack([x if x is not None else np.zeros(shape, np.float32) for x in imgs])
    starts = [-1 if idx == -1 else clips[idx][0] for idx in window_indices]
    return img_clips, ids, masks, 1 if is_positive else 0, starts, image_num, target_idx, len(clips)
