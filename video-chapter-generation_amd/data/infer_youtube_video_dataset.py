"""Drop-in for reference data/infer_youtube_video_dataset.py `InferYoutubeClipDataset` (:218-313): the eval
dataset over the pre-flattened clip JSON (video_chapter_youtube_dataset/flat_video2clip_for_quick_infer.py; written
here by data.clip_windows.video_clip_infos). Same constructor and sample tuple:

    InferYoutubeClipDataset(img_dir, json_paths, tokenizer, clip_frame_num, max_text_len, mode="all",
                            transform=None, target_transform=None)
    item i -> (img_clip f32 [T, 3, H, W] (0 in text mode), text_ids i64 [L], attention_mask i64 [L], clip_label)

json_paths: one JSON file or a list of them (records concatenated in order); `all_clip_infos` is the record
list the trainers write `pred_score` into. Frames are the records' `image_paths`, decoded with PIL -> RGB ->
`transform`; `u8=True` returns the u8 [T, H, W, 3] stack for the GPU ingest kernel instead.
"""
import json

import torch

from . import clip_windows as cw
from .youtube_dataset import frames_tensor


class InferYoutubeClipDataset(torch.utils.data.Dataset):
    def __init__(self, img_dir, json_paths, tokenizer, clip_frame_num, max_text_len, mode="all", transform=None,
                 target_transform=None, u8=False):
        self.max_offset = 2
        self.tokenizer = tokenizer
        self.clip_frame_num = clip_frame_num
        self.max_text_len = max_text_len
        self.mode = mode
        self.half_clip_frame_num = int(clip_frame_num // 2)
        self.img_dir = img_dir
        if isinstance(json_paths, (list, tuple)):
            self.all_clip_infos = []
            for p in json_paths:
                with open(p, "r", encoding="utf-8") as f:
                    self.all_clip_infos.extend(json.load(f))
        else:
            with open(json_paths) as f:
                self.all_clip_infos = json.load(f)
        self.transform = transform
        self.target_transform = target_transform
        self.u8 = u8

    def __len__(self):
        return len(self.all_clip_infos)

    def __getitem__(self, i):
        info = self.all_clip_infos[i]
        ids, mask = cw.encode_text(self.tokenizer, info["text_clip"], self.max_text_len)
        img_clip = 0 if self.mode == "text" else frames_tensor(info["image_paths"], self.transform, self.u8)
        return img_clip, torch.from_numpy(ids), torch.from_numpy(mask), info["clip_label"]
