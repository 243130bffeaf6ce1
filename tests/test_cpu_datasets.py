"""The disk-backed datasets with the reference's signatures (data/youtube_dataset.py, data/
infer_youtube_video_dataset.py, data/common_utils.py) on a synthetic corpus written to tmp in the reference's
on-disk formats: dataset CSV ("%^&*"-joined timestamps), vid list, <dir>/<vid>/subtitle_<vid>.json, and
<img_dir>/<vid>/%05d.jpg frames (PIL JPEG). Checked against oracle/windows.py's statement-by-statement restatement
of YoutubeClipDataset.__getitem__ (youtube_dataset.py:64-194), with transformers.BertTokenizer -- the reference's
tokenizer class -- on a synthetic vocab file (bert-base-uncased's vocab cannot be fetched here)."""
import json
import os
import random

import numpy as np
import pytest
import torch


from corpus_util import tokenizer as _tokenizer
from corpus_util import write_corpus as _write_corpus


def test_parse_csv_to_list(tmp_path):
    from data.common_utils import parse_csv_to_list
    img_dir, data_file, vid_file, subs, ts, _ = _write_corpus(str(tmp_path))
    vids, titles, durations, timestamps = parse_csv_to_list(data_file)
    assert vids == ["vid00XyZ", "vid01XyZ"] and titles == ["title vid00XyZ", "title vid01XyZ"]
    assert durations == [40.5, 57.5] and timestamps == ts


@pytest.mark.parametrize("seed", [1, 2, 3, 4])
def test_youtube_clip_dataset_matches_reference_restatement(tmp_path, seed):
    from data.clip_windows import extract_first_timestamp
    from data.transforms import train_vision_preprocess
    from data.youtube_dataset import YoutubeClipDataset
    from oracle.windows import youtube_clip_item
    img_dir, data_file, vid_file, subs, ts, vocab = _write_corpus(str(tmp_path))
    tok = _tokenizer(vocab)
    ds = YoutubeClipDataset(img_dir, data_file, vid_file, tok, 16, 24, transform=train_vision_preprocess())
    assert len(ds) == 2
    for i, vid in enumerate(ds.vids):
        random.seed(seed)
        torch.manual_seed(seed)
        img, ids, mask, label = ds[i]
        rng = random.Random(seed)
        exp_img, exp_ids, exp_mask, exp_label, _ = youtube_clip_item(
            img_dir, vid, [extract_first_timestamp(t)[0] for t in ts[i]], subs[vid], tok, 16, 24, rng)
        assert label == exp_label
        assert ids.tolist() == list(exp_ids) and mask.tolist() == list(exp_mask)
        assert img.shape == (16, 3, 32, 32) and img.dtype == torch.float32
        assert np.array_equal(img.numpy(), exp_img)
    # u8 mode: the decoded frames, for the GPU ingest kernel (normalised there)
    ds8 = YoutubeClipDataset(img_dir, data_file, vid_file, tok, 16, 24, u8=True)
    random.seed(seed)
    img8, _, _, _ = ds8[0]
    random.seed(seed)
    imgf, _, _, _ = ds[0]
    assert img8.dtype == torch.uint8 and img8.shape == (16, 32, 32, 3)
    ref = (img8.float() / 255.0 - torch.tensor([0.485, 0.456, 0.406])) / torch.tensor([0.229, 0.224, 0.225])
    assert torch.equal(ref.permute(0, 3, 1, 2), imgf)


def test_infer_dataset_reads_clip_json(tmp_path):
    from data.clip_windows import video_clip_infos
    from data.infer_youtube_video_dataset import InferYoutubeClipDataset
    from data.transforms import test_vision_preprocess
    from oracle.windows import frame_numbers
    img_dir, data_file, vid_file, subs, ts, vocab = _write_corpus(str(tmp_path))
    tok = _tokenizer(vocab)
    paths = []
    for v, (vid, n) in enumerate(zip(["vid00XyZ", "vid01XyZ"], (40, 57))):
        recs = video_clip_infos(vid, img_dir, n, ts[v], subs[vid], 16)
        p = os.path.join(str(tmp_path), f"clips_{v}.json")
        with open(p, "w") as f:
            json.dump(recs, f)
        paths.append(p)
    ds = InferYoutubeClipDataset(img_dir, paths, tok, 16, 24, transform=test_vision_preprocess())
    assert len(ds) == len(ds.all_clip_infos) > 0
    from PIL import Image
    for i in (0, len(ds) // 2, len(ds) - 1):
        info = ds.all_clip_infos[i]
        img, ids, mask, label = ds[i]
        s, e = info["clip_start_end"]
        n = 40 if info["vid"] == "vid00XyZ" else 57
        assert [int(os.path.basename(p)[:5]) for p in info["image_paths"]] == frame_numbers(s, e, n, 16)
        with Image.open(info["image_paths"][3]) as im:
            a = np.asarray(im.convert("RGB"), dtype=np.float32) / np.float32(255.0)
        exp = ((a - np.array([0.485, 0.456, 0.406], np.float32)) / np.array([0.229, 0.224, 0.225], np.float32))
        assert np.array_equal(img[3].numpy(), exp.transpose(2, 0, 1))
        toks = tok.tokenize("[CLS] " + info["text_clip"])[:24]
        assert ids.tolist()[:len(toks)] == tok.convert_tokens_to_ids(toks) and int(mask.sum()) == len(toks)
        assert label == info["clip_label"]
    text_ds = InferYoutubeClipDataset(img_dir, paths[0], tok, 16, 24, mode="text")
    assert text_ds[0][0] == 0


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_window_clip_dataset_matches_reference_restatement(tmp_path, seed):
    from data.clip_windows import extract_first_timestamp
    from data.transforms import train_vision_preprocess
    from data.youtube_dataset import WindowClipDataset
    from oracle.windows import window_clip_item
    img_dir, data_file, vid_file, subs, ts, vocab = _write_corpus(str(tmp_path))
    tok = _tokenizer(vocab)
    ds = WindowClipDataset(img_dir, data_file, vid_file, tok, 8, 24, window_size=2, transform=train_vision_preprocess())
    for i, vid in enumerate(ds.vids):
        random.seed(seed + i)
        torch.manual_seed(seed)
        img, ids, mask, label, info = ds[i]
        rng = random.Random(seed + i)
        exp = window_clip_item(img_dir, vid, [extract_first_timestamp(t)[0] for t in ts[i]], subs[vid], tok, 8, 24, 2, rng)
        e_img, e_ids, e_mask, e_label, starts, image_num, target, n_clips = exp
        assert int(label) == e_label
        assert ids.tolist() == [list(x) for x in e_ids] and mask.tolist() == e_mask
        assert img.shape == (5, 8, 3, 32, 32) and np.array_equal(img.numpy(), e_img)
        assert info["clip_start_frame"].tolist() == starts
        assert int(info["total_frames"]) == image_num and int(info["target_clip_idx"]) == target
        assert int(info["total_num_clips"]) == n_clips


def test_synthetic_corpus_round_trips_through_disk(tmp_path):
    """SyntheticVideoCorpus.write -> the reference-format tree; YoutubeClipDataset over it returns the corpus's own
    frames (JPEG-decoded) for the sampled window."""
    from data.synthetic_dataset import HashTokenizer, SyntheticVideoCorpus
    from data.youtube_dataset import YoutubeClipDataset
    c = SyntheticVideoCorpus(2, 30, 40, H=32, W=32, seed=4)
    img_dir, data_file, vid_file = c.write(str(tmp_path))
    ds = YoutubeClipDataset(img_dir, data_file, vid_file, HashTokenizer(), 8, 16, u8=True)
    random.seed(0)
    img, ids, mask, label = ds[1]
    assert img.shape == (8, 32, 32, 3) and img.dtype == torch.uint8
    assert len(os.listdir(os.path.join(img_dir, c.vids[1]))) == c.image_num[c.vids[1]]
