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
