"""Drop-ins for reference data/youtube_dataset.py `YoutubeClipDataset` (:23-194) and `WindowClipDataset`
(:359-536, the window model's sampler): training samplers over videos on disk. Same constructor, same sample tuple, same index / label / text / frame-file rules:

    YoutubeClipDataset(img_dir, data_file, vid_file, tokenizer, clip_frame_num, max_text_len, mode="all",
                       transform=None, target_transform=None, subtitle_dir=None)
    item i -> (img_clip f32 [T, 3, H, W] (0 in text mode), text_ids i64 [L], attention_mask i64 [L], label)

- data_file: the dataset CSV (data.common_utils.parse_csv_to_list); vid_file: one video id per line;
- subtitles: <subtitle_dir or dirname(data_file)>/*/subtitle_<vid>.json (list of {"start", "text"});
- frames: <img_dir>/<vid>/%05d.jpg at 1 fps, counted by glob (`image_num`), decoded with PIL -> RGB ->
  `transform` (the reference passes ToTensor + Normalize, data/transforms.py);
- item i samples a positive window with probability 1/2 when the video has one, else a negative (Python
  `random`, as the reference), windows [s, s + T) every 2 * max_offset = 4 s, IoU labels, frame files +1 near
  the ends / +3 elsewhere, subtitles in (s - 1, e + 1), "[CLS] " + text tokenised, truncated, [PAD]-padded
  (data/clip_windows.py holds the restated rules, each citing its reference lines).

`u8=True` (MI355X ingest): img_clip is the decoded u8 [T, H, W, 3] stack instead, for vcg_window_frames_u8 to
gather + normalise on the GPU (`transform` is then not applied).
"""
import glob
import json
import os
import random

import numpy as np
import torch

from . import clip_windows as cw
from .common_utils import parse_csv_to_list


def load_frame(path):
    from PIL import Image
    with Image.open(path) as im:
        return im.convert("RGB")


def subtitle_files(subtitle_path):
    """{vid: path} of <subtitle_path>/*/subtitle_<vid>.json (youtube_dataset.py:50-57)."""
    out = {}
    for f in glob.glob(subtitle_path + "/*/subtitle_*.json"):
        out[os.path.basename(f).split(".")[0][9:]] = f
    return out


def frames_tensor(paths, transform, u8):
    imgs = [load_frame(p) for p in paths]
    if u8:
        return torch.from_numpy(np.stack([np.asarray(im, dtype=np.uint8) for im in imgs]))
    if transform is None:
        raise ValueError("transform is required unless u8=True (the reference always passes one)")
    return torch.stack([transform(im) for im in imgs], dim=0)


class YoutubeClipDataset(torch.utils.data.Dataset):
    def __init__(self, img_dir, data_file, vid_file, tokenizer, clip_frame_num, max_text_len, mode="all",
                 transform=None, target_transform=None, subtitle_dir=None, u8=False):
        self.tokenizer = tokenizer
        self.clip_frame_num = clip_frame_num
        self.max_text_len = max_text_len
        self.mode = mode
        self.half_clip_frame_num = int(clip_frame_num // 2)
        self.img_dir = img_dir
        vids, titles, durations, timestamps = parse_csv_to_list(data_file)
        self.vid2title = dict(zip(vids, titles))
        self.vid2timestamps = dict(zip(vids, timestamps))
        self.vid2durations = dict(zip(vids, durations))
        with open(vid_file) as f:
            self.vids = [x.strip() for x in f.readlines()]
        self.vid2asr_files = subtitle_files(os.path.dirname(data_file) if subtitle_dir is None else subtitle_dir)
        self.transform = transform
        self.target_transform = target_transform
        self.u8 = u8

    def __len__(self):
        return len(self.vids)

    def __getitem__(self, i):
        vid = self.vids[i]
        image_path = os.path.join(self.img_dir, vid)
        image_num = len(glob.glob(image_path + "/*.jpg"))
        with open(self.vid2asr_files[vid]) as f:
            subtitles = json.load(f)
        cut_points = cw.cut_points_from_timestamps(self.vid2timestamps[vid], image_num, mode="train")
        win = cw.clip_windows(image_num, self.clip_frame_num)
        if len(win) == 0:
            raise ValueError(f"video {vid}: {image_num} frames is shorter than one clip")
        labels = cw.clip_labels(win, cut_points, self.clip_frame_num)
        pos = np.nonzero(labels == 1)[0].tolist()
        neg = np.nonzero(labels == 0)[0].tolist()
        is_positive = 0 if not pos else random.sample([0, 1], k=1)[0]   # youtube_dataset.py:124-133
        k = random.sample(pos, k=1)[0] if is_positive else random.sample(neg, k=1)[0]
        s, e = win[k].tolist()
        ids, mask = cw.encode_text(self.tokenizer, cw.window_text(subtitles, s, e), self.max_text_len)
        if self.mode == "text":
            img_clip = 0
        else:
            nums = cw.frame_numbers(s, self.clip_frame_num, image_num)
            img_clip = frames_tensor([os.path.join(image_path, "%05d.jpg" % n) for n in nums.tolist()],
                                     self.transform, self.u8)
        return img_clip, torch.from_numpy(ids), torch.from_numpy(mask), 1 if is_positive else 0


class WindowClipDataset(torch.utils.data.Dataset):
    """Reference youtube_dataset.py:359-536: item i = a positive / negative target clip of video i with its window of
    2 * window_size + 1 clips `T // (2 * max_offset)` clips apart (-1 off the video ends -> zero padding clip):

        (img_clips f32 [2w+1, T, 3, H, W] (tensor(0) in text mode), text_ids i64 [2w+1, L],
         attention_masks i64 [2w+1, L], label, clip_info)

    clip_info = {clip_start_frame [2w+1] (-1 padding), total_frames, target_clip_idx, total_num_clips}. Differences
    from YoutubeClipDataset that the reference has and this keeps: cut points kept for 4 <= sec <= N - 4 (:399-402),
    random.choice draws (:428-429), the window text "[CLS] " + every subtitle text followed by a space (:480-483),
    padding clips of zero frames at the real frame size (the reference hard-codes 224x224, :451)."""

    def __init__(self, img_dir, data_file, vid_file, tokenizer, clip_frame_num, max_text_len, window_size=2,
                 mode="all", transform=None, subtitle_dir=None, u8=False):
        self.tokenizer = tokenizer
        self.clip_frame_num = clip_frame_num
        self.max_text_len = max_text_len
        self.window_size = window_size
        self.mode = mode
        self.half_clip_frame_num = int(clip_frame_num // 2)
        self.img_dir = img_dir
        self.fps = 1
        vids, titles, durations, timestamps = parse_csv_to_list(data_file)
        self.vid2title = dict(zip(vids, titles))
        self.vid2timestamps = dict(zip(vids, timestamps))
        self.vid2durations = dict(zip(vids, durations))
        with open(vid_file) as f:
            self.vids = [x.strip() for x in f.readlines()]
        self.vid2asr_files = subtitle_files(os.path.dirname(data_file) if subtitle_dir is None else subtitle_dir)
        self.transform = transform
        self.u8 = u8

    def __len__(self):
        return len(self.vids)

    def __getitem__(self, i):
        vid = self.vids[i]
        image_path = os.path.join(self.img_dir, vid)
        image_num = len(glob.glob(image_path + "/*.jpg"))
        with open(self.vid2asr_files[vid]) as f:
            subtitles = json.load(f)
        T, L = self.clip_frame_num, self.max_text_len
        cut_points = cw.cut_points_from_timestamps(self.vid2timestamps[vid], image_num, mode="eval", fps=self.fps)
        max_offset = 2 * self.fps
        win = cw.clip_windows(image_num, T, max_offset)
        labels = cw.clip_labels(win, cut_points, T, max_offset)
        pos = np.nonzero(labels == 1)[0].tolist()
        neg = np.nonzero(labels == 0)[0].tolist()
        is_positive = random.choice([0, 1]) if pos else 0
        target = random.choice(pos if is_positive else neg)
        idx = cw.window_clip_indices(target, len(win), T, self.window_size, max_offset)
        imgs, ids, masks = [], [], []
        pad_shape = None
        for k in idx:
            if k < 0:
                ids.append(torch.zeros(L, dtype=torch.long))
                masks.append(torch.zeros(L, dtype=torch.long))
                imgs.append(None)
                continue
            s, e = win[k].tolist()
            text = "[CLS] " + "".join(sub["text"] + " " for sub in subtitles
                                      if s - self.fps < sub["start"] < e + self.fps)
            tokens = self.tokenizer.tokenize(text)[:L]
            n = len(tokens)
            tokens = tokens + ["[PAD]"] * (L - n)
            ids.append(torch.tensor(self.tokenizer.convert_tokens_to_ids(tokens), dtype=torch.long))
            masks.append(torch.tensor([1] * n + [0] * (L - n), dtype=torch.long))
            if self.mode != "text":
                nums = cw.frame_numbers(s, T, image_num)
                clip = frames_tensor([os.path.join(image_path, "%05d.jpg" % f) for f in nums.tolist()], self.transform,
                                     self.u8)
                pad_shape = (clip.shape, clip.dtype)
                imgs.append(clip)
        if self.mode == "text":
            img_clips = torch.tensor(0)
        else:
            img_clips = torch.stack([c if c is not None else torch.zeros(*pad_shape[0], dtype=pad_shape[1])
                                     for c in imgs])
        info = cw.window_clip_info(win, target, T, self.window_size, image_num, max_offset)
        clip_info = {k: torch.as_tensor(v) for k, v in info.items()}
        return img_clips, torch.stack(ids), torch.stack(masks), torch.tensor(1 if is_positive else 0), clip_info
