"""Synthetic stand-ins for the reference's datasets. There is no network here, so there are no YouTube
frames, subtitles or bert-base-uncased vocab files. The classes produce the same sample tuples
`(img_clip f32 [T,3,H,W], text_ids i64 [L], attention_mask i64 [L], label)` through the real
window / label / frame-index / subtitle logic (`data/clip_windows.py`):

- `SyntheticVideoCorpus`: videos with chapter timestamps, subtitles and deterministic u8 frames.
- `YoutubeClipDataset`: the training sampler (`data/youtube_dataset.py:23-194`). For each video it
  draws a positive or a negative window with Python `random`, as the reference does.
- `InferYoutubeClipDataset`: the eval dataset over clip-JSON records
  (`data/infer_youtube_video_dataset.py:229-300`). The records can be read from a JSON file
  written by `data.clip_windows.video_clip_infos`.
- `HashTokenizer`: a whitespace tokenizer with hashed ids, used when no BERT vocab is available.
"""
import json
import random

import numpy as np
import torch

from vcg_hip import synth
from . import clip_windows as cw

MEAN = np.array([0.485, 0.456, 0.406], dtype=np.float32)
STD = np.array([0.229, 0.224, 0.225], dtype=np.float32)


class HashTokenizer:
    """`tokenize` splits on whitespace (lower-cased, "[CLS]"/"[PAD]" kept). `convert_tokens_to_ids`
    maps [PAD] -> 0 and [CLS] -> 101. Any other token gets an FNV-1a hash in [1000, vocab)."""

    def __init__(self, vocab_size=30522):
        self.vocab_size = vocab_size

    def tokenize(self, text):
        return [t if t in ("[CLS]", "[PAD]") else t.lower() for t in text.split()]

    def convert_tokens_to_ids(self, tokens):
        out = []
        for t in tokens:
            if t == "[PAD]":
                out.append(0)
            elif t == "[CLS]":
                out.append(101)
            else:
                h = 0xCBF29CE484222325
                for b in t.encode():
                    h = ((h ^ b) * 0x100000001B3) & 0xFFFFFFFFFFFFFFFF
                out.append(1000 + h % (self.vocab_size - 1000))
        return out


def normalize_frames(u8):
    """u8 [..., H, W, 3] -> f32 [..., 3, H, W] as ToTensor + Normalize (fp32)."""
    x = torch.from_numpy(np.ascontiguousarray(u8)).float() / 255.0
    x = (x - torch.from_numpy(MEAN)) / torch.from_numpy(STD)
    return x.movedim(-1, -3).contiguous()


class SyntheticVideoCorpus:
    """`n_videos` videos at 1 fps. Each video has a length in [min_len, max_len] seconds, a chapter
    about every `chapter_every` s and a subtitle about every 3 s. Frame f of video v is u8
    [H,W,3] noise keyed by (seed, v, f), so any frame can be rebuilt anywhere."""

    def __init__(self, n_videos=4, min_len=60, max_len=200, chapter_every=40, H=112, W=112, seed=123):
        rng = random.Random(seed)
        self.H, self.W, self.seed = H, W, seed
        self.vids, self.image_num, self.timestamps, self.subtitles = [], {}, {}, {}
        for v in range(n_videos):
            vid = f"synvid{v:04d}"
            n = rng.randint(min_len, max_len)
            self.vids.append(vid)
            self.image_num[vid] = n
            t, ts = 0, []
            while t < n:
                ts.append(f"{t // 60}:{t % 60:02d} chapter {len(ts)}")
                t += max(5, int(rng.gauss(chapter_every, chapter_every / 4)))
            self.timestamps[vid] = ts
            subs, s = [], 0.0
            while s < n:
                subs.append({"start": round(s, 2), "text": " ".join(f"w{rng.randint(0, 500)}" for _ in range(rng.randint(1, 6)))})
                s += rng.uniform(1.0, 5.0)
            self.subtitles[vid] = subs

    def frames(self, vid, frame_indices):
        """u8 [len(frame_indices), H, W, 3] for 0-based frame indices."""
        out = np.empty((len(frame_indices), self.H, self.W, 3), dtype=np.uint8)
        for k, f in enumerate(frame_indices):
            key = synth.key_of(self.seed, f"{vid}/frame{int(f)}")
            out[k] = synth.fill_np(self.H * self.W * 3, synth.KIND_INT, key, 0, 256).astype(np.uint8).reshape(
                self.H, self.W, 3)
        return out

    def all_frames(self, vid):
        return self.frames(vid, range(self.image_num[vid]))

    def write(self, root, split_name="train.txt", quality=95):
        """Write the corpus in the reference's on-disk layout (the inputs of data/youtube_dataset.py's datasets):
        <root>/frames/<vid>/%05d.jpg (1-based, PIL JPEG), <root>/subtitles/<vid>/subtitle_<vid>.json, the dataset
        CSV <root>/subtitles/data.csv ("%^&*"-joined timestamps) and the vid list <root>/<split_name>.
        Returns (img_dir, data_file, vid_file)."""
        import os

        from PIL import Image

        from .common_utils import write_csv
        img_dir = os.path.join(root, "frames")
        sub_dir = os.path.join(root, "subtitles")
        for vid in self.vids:
            d = os.path.join(img_dir, vid)
            os.makedirs(d, exist_ok=True)
            for f, fr in enumerate(self.all_frames(vid)):
                Image.fromarray(fr).save(os.path.join(d, "%05d.jpg" % (f + 1)), quality=quality)
            sd = os.path.join(sub_dir, vid)
            os.makedirs(sd, exist_ok=True)
            with open(os.path.join(sd, f"subtitle_{vid}.json"), "w") as fh:
                json.dump(self.subtitles[vid], fh)
        data_file = os.path.join(sub_dir, "data.csv")
        write_csv(data_file, self.vids, [f"synthetic {v}" for v in self.vids],
                  [float(self.image_num[v]) for v in self.vids], [self.timestamps[v] for v in self.vids])
        vid_file = os.path.join(root, split_name)
        with open(vid_file, "w") as fh:
            fh.write("\n".join(self.vids) + "\n")
        return img_dir, data_file, vid_file


def _encode(tokenizer, text, max_text_len):
    ids, mask = cw.encode_text(tokenizer, text, max_text_len)
    return torch.from_numpy(ids), torch.from_numpy(mask)


class YoutubeClipDataset(torch.utils.data.Dataset):
    """Training sampler: item i is a random positive or negative window of video i."""

    def __init__(self, corpus, tokenizer, clip_frame_num, max_text_len, mode="all"):
        self.c, self.tok, self.T, self.L, self.mode = corpus, tokenizer, clip_frame_num, max_text_len, mode

    def __len__(self):
        return len(self.c.vids)

    def __getitem__(self, i):
        vid = self.c.vids[i]
        n = self.c.image_num[vid]
        cps = cw.cut_points_from_timestamps(self.c.timestamps[vid], n, mode="train")
        win = cw.clip_windows(n, self.T)
        lab = cw.clip_labels(win, cps, self.T)
        pos = np.nonzero(lab == 1)[0].tolist()
        neg = np.nonzero(lab == 0)[0].tolist()
        is_pos = 0 if not pos else random.sample([0, 1], k=1)[0]      # youtube_dataset.py:119-131
        k = random.sample(pos, k=1)[0] if is_pos else random.sample(neg, k=1)[0]
        s, e = win[k].tolist()
        ids, mask = _encode(self.tok, cw.window_text(self.c.subtitles[vid], s, e), self.L)
        img = 0 if self.mode == "text" else normalize_frames(self.c.frames(vid, cw.frame_numbers(s, self.T, n) - 1))
        return img, ids, mask, int(is_pos)


class InferYoutubeClipDataset(torch.utils.data.Dataset):
    """Eval dataset over clip records (all windows of every video, stride 4 s)."""

    max_offset = 2

    def __init__(self, corpus, tokenizer, clip_frame_num, max_text_len, mode="all", json_path=None):
        self.c, self.tok, self.T, self.L, self.mode = corpus, tokenizer, clip_frame_num, max_text_len, mode
        if json_path is not None:
            with open(json_path) as f:
                self.all_clip_infos = json.load(f)
        else:
            self.all_clip_infos = []
            for vid in corpus.vids:
                self.all_clip_infos += cw.video_clip_infos(vid, "synthetic", corpus.image_num[vid],
                                                           corpus.timestamps[vid], corpus.subtitles[vid],
                                                           clip_frame_num)

    def __len__(self):
        return len(self.all_clip_infos)

    def __getitem__(self, i):
        info = self.all_clip_infos[i]
        ids, mask = _encode(self.tok, info["text_clip"], self.L)
        if self.mode == "text":
            img = 0
        else:
            nums = [int(p.rsplit("/", 1)[-1].split(".")[0]) for p in info["image_paths"]]
            img = normalize_frames(self.c.frames(info["vid"], [x - 1 for x in nums]))
        return img, ids, mask, info["clip_label"]
