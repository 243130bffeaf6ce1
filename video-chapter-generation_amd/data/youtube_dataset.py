"""Drop-in for reference data/youtube_dataset.py `YoutubeClipDataset` (:23-194): the training sampler over
videos on disk. Same constructor, same sample tuple, same index / label / text / frame-file rules:

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
