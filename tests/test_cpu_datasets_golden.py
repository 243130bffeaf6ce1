"""The drop-in datasets against outputs of the REFERENCE's own dataset classes (row a10): tests/golden/datasets.json
was written by tools/oracle/make_golden_datasets.py, which runs the reference's YoutubeClipDataset,
WindowClipDataset (youtube_dataset.py:23-197, :359-539) and InferYoutubeClipDataset
(infer_youtube_video_dataset.py:218-313) -- unmodified, ast-extracted -- over tests/corpus_util.py's corpus with
the same tokenizer, transform and seeds. Token ids, masks, labels, clips_info and image digests must be equal."""
import json
import os
import random

import pytest
import torch

import corpus_util as cu

GOLD = os.path.join(os.path.dirname(__file__), "golden", "datasets.json")


@pytest.fixture(scope="module")
def corpus(tmp_path_factory):
    with open(GOLD) as f:
        gold = json.load(f)
    root = str(tmp_path_factory.mktemp("corpus"))
    img_dir, data_file, vid_file, subs, ts, vocab = cu.write_corpus(root, hw=gold["hw"])
    return gold, root, img_dir, data_file, vid_file, subs, ts, cu.tokenizer(vocab)


def _seeded(seed):
    random.seed(seed)
    torch.manual_seed(seed)


def test_youtube_clip_dataset_equals_reference_run(corpus):
    from data.transforms import train_vision_preprocess
    from data.youtube_dataset import YoutubeClipDataset
    gold, root, img_dir, data_file, vid_file, subs, ts, tok = corpus
    g = gold["youtube_clip"]
    ds = YoutubeClipDataset(img_dir, data_file, vid_file, tok, g["clip_frame_num"], g["max_text_len"],
                            transform=train_vision_preprocess())
    for it in g["items"]:
        _seeded(it["seed"])
        img, ids, mask, label = ds[it["i"]]
        assert (int(label), ids.tolist(), mask.tolist()) == (it["label"], it["ids"], it["mask"]), it
        assert list(img.shape) == it["img_shape"] and cu.tensor_digest(img.numpy()) == it["img"], it


def test_window_clip_dataset_equals_reference_run(corpus):
    from data.transforms import train_vision_preprocess
    from data.youtube_dataset import WindowClipDataset
    gold, root, img_dir, data_file, vid_file, subs, ts, tok = corpus
    g = gold["window_clip"]
    padded = 0
    for mode in ("all", "text"):
        ds = WindowClipDataset(img_dir, data_file, vid_file, tok, g["clip_frame_num"], g["max_text_len"],
                               window_size=g["window_size"], mode=mode, transform=train_vision_preprocess())
        for it in (x for x in g["items"] if x["mode"] == mode):
            _seeded(it["seed"])
            img, ids, mask, label, info = ds[it["i"]]
            assert (int(label), ids.tolist(), mask.tolist()) == (it["label"], it["ids"], it["mask"]), it
            assert {k: v.tolist() for k, v in info.items()} == it["info"], it
            assert list(img.shape) == it["img_shape"] and cu.tensor_digest(img.numpy()) == it["img"], it
            padded += -1 in it["info"]["clip_start_frame"]
    assert padded > 0  # the zero-padding clips (window running off the video) are covered


def test_infer_clip_dataset_equals_reference_run(corpus):
    from data.infer_youtube_video_dataset import InferYoutubeClipDataset
    from data.transforms import train_vision_preprocess
    gold, root, img_dir, data_file, vid_file, subs, ts, tok = corpus
    g = gold["infer_clip"]
    paths = cu.write_clip_jsons(root, img_dir, subs, ts, g["clip_frame_num"])
    ds = InferYoutubeClipDataset(img_dir, paths, tok, g["clip_frame_num"], g["max_text_len"],
                                 transform=train_vision_preprocess())
    assert len(ds) == g["n"]
    for it in g["items"]:
        _seeded(it["i"])
        img, ids, mask, label = ds[it["i"]]
        assert (int(label), ids.tolist(), mask.tolist()) == (it["label"], it["ids"], it["mask"]), it
        assert list(img.shape) == it["img_shape"] and cu.tensor_digest(img.numpy()) == it["img"], it
