"""A small corpus in the reference's on-disk dataset format, written deterministically (test helper; also used by
tools/oracle/make_golden_datasets.py, which runs the REFERENCE dataset classes over the same files):

    <root>/frames/<vid>/%05d.jpg            frames at 1 fps (PIL JPEG, quality 95)
    <root>/subs/<vid>/subtitle_<vid>.json   [{"start": sec, "text": ...}, ...]
    <root>/subs/data.csv                    vid, title, duration, "%^&*"-joined chapter timestamps
    <root>/train.txt                        one vid per line
    <root>/vocab.txt                        a BERT WordPiece vocab for transformers.BertTokenizer
"""
import hashlib
import json
import os

import numpy as np

N_FRAMES = (40, 57)
VIDS = ("vid00XyZ", "vid01XyZ")


def write_corpus(root, n_videos=2, n_frames=N_FRAMES, hw=32, seed=0):
    from PIL import Image
    from data.common_utils import write_csv
    rng = np.random.default_rng(seed)
    words = [f"word{i}" for i in range(50)] + ["hello", "world", "chapter", "intro"]
    vids, timestamps, subs = [], [], {}
    for v in range(n_videos):
        vid = f"vid{v:02d}XyZ"
        vids.append(vid)
        d = os.path.join(root, "frames", vid)
        os.makedirs(d)
        for f in range(n_frames[v]):
            Image.fromarray(rng.integers(0, 256, (hw, hw, 3), dtype=np.uint8)).save(os.path.join(d, "%05d.jpg" % (f + 1)),
                                                                                    quality=95)
        timestamps.append([f"0:{t // 60:02d}:{t % 60:02d} part {k}" if t >= 60 else f"{t // 60}:{t % 60:02d} part {k}"
                           for k, t in enumerate([0, 9, 21, n_frames[v] - 6])])
        sd = os.path.join(root, "subs", vid)
        os.makedirs(sd)
        subs[vid] = [{"start": round(float(s), 2), "text": " ".join(rng.choice(words, size=rng.integers(1, 6)))}
                     for s in np.arange(0.0, n_frames[v], 2.7)]
        with open(os.path.join(sd, f"subtitle_{vid}.json"), "w") as f:
            json.dump(subs[vid], f)
    data_file = os.path.join(root, "subs", "data.csv")
    write_csv(data_file, vids, [f"title {v}" for v in vids], [n + 0.5 for n in n_frames], timestamps)
    vid_file = os.path.join(root, "train.txt")
    with open(vid_file, "w") as f:
        f.write("\n".join(vids) + "\n")
    vocab = os.path.join(root, "vocab.txt")
    with open(vocab, "w") as f:
        f.write("\n".join(["[PAD]"] + [f"[unused{i}]" for i in range(99)] + ["[UNK]", "[CLS]", "[SEP]", "[MASK]"]
                          + words + ["##1", "##2", "word", "part"]) + "\n")
    return os.path.join(root, "frames"), data_file, vid_file, subs, timestamps, vocab


def tokenizer(vocab):
    from transformers import BertTokenizer
    return BertTokenizer(vocab_file=vocab, do_lower_case=True)


def write_clip_jsons(root, img_dir, subs, timestamps, clip_frame_num=16):
    """flat_video2clip_for_quick_infer-format clip lists (data.clip_windows.video_clip_infos), one file per video
    (absolute image paths; the goldens record only what a dataset returns, never a path)."""
    from data.clip_windows import video_clip_infos
    paths = []
    for v, (vid, n) in enumerate(zip(VIDS, N_FRAMES)):
        recs = video_clip_infos(vid, img_dir, n, timestamps[v], subs[vid], clip_frame_num)
        p = os.path.join(root, f"clips_{v}.json")
        with open(p, "w") as f:
            json.dump(recs, f)
        paths.append(p)
    return paths


def tensor_digest(x):
    """sha256 of a tensor's (shape, dtype, C-order bytes): images are pinned by digest, not stored."""
    a = np.ascontiguousarray(np.asarray(x))
    h = hashlib.sha256()
    h.update(repr((a.shape, str(a.dtype))).encode())
    h.update(a.tobytes())
    return h.hexdigest()
