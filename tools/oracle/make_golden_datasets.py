"""Generate tests/golden/datasets.json: outputs of the REFERENCE dataset classes, run here (row a10).

Runs only in the build container (it reads /root/reference). The reference modules
`data/youtube_dataset.py` and `data/infer_youtube_video_dataset.py` cannot be imported whole here: their
module-level imports name torchvision and matplotlib, which this image lacks, and neither is used by the classes
pinned below. So the script parses each module with `ast` and executes only the class definitions
`YoutubeClipDataset` (:23-197), `WindowClipDataset` (:359-539) and `InferYoutubeClipDataset` (:218-313) -- the
reference's own code, unmodified -- in a namespace holding the real modules those classes use (torch, numpy, glob,
random, os, json, PIL.Image) and the reference's own `data/common_utils.py` functions (loaded by path). Nothing is
stubbed.

Inputs: the corpus of tests/corpus_util.py (224x224 JPEG frames, so the window dataset's hard-coded
(T, 3, 224, 224) zero padding stacks), transformers.BertTokenizer on the corpus's synthetic vocab (the reference's
tokenizer class; bert-base-uncased's vocab cannot be fetched), and data.transforms.train_vision_preprocess() as
the `transform` argument (the restated torchvision pipeline: the golden pins the dataset logic, not torchvision).
Python's `random` and torch's RNG are seeded before each item, as the tests do. Images are pinned by sha256 digest.

Usage: python tools/oracle/make_golden_datasets.py
"""
import ast
import importlib.util
import glob
import json
import os
import random
import sys
import tempfile

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference/video_chapter_generation"
for p in (os.path.join(REPO, "video-chapter-generation_amd"), os.path.join(REPO, "tests"), REPO):
    sys.path.insert(0, p)

HW = 224


def ref_classes(module_file, names):
    spec = importlib.util.spec_from_file_location("ref_common_utils", os.path.join(REF, "data", "common_utils.py"))
    cu = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(cu)
    from PIL import Image
    ns = {"torch": torch, "np": np, "glob": glob, "random": random, "os": os, "json": json, "Image": Image,
          "parse_csv_to_list": cu.parse_csv_to_list, "extract_first_timestamp": cu.extract_first_timestamp}
    path = os.path.join(REF, "data", module_file)
    with open(path) as f:
        tree = ast.parse(f.read(), filename=path)
    nodes = [n for n in tree.body if isinstance(n, ast.ClassDef) and n.name in names]
    assert sorted(n.name for n in nodes) == sorted(names), [n.name for n in nodes]
    exec(compile(ast.Module(body=nodes, type_ignores=[]), path, "exec"), ns)
    return [ns[n] for n in names]


def seeded(seed):
    random.seed(seed)
    torch.manual_seed(seed)


def main():
    import corpus_util as cu
    from data.transforms import train_vision_preprocess
    YoutubeClipDataset, WindowClipDataset = ref_classes("youtube_dataset.py",
                                                        ["YoutubeClipDataset", "WindowClipDataset"])
    (InferYoutubeClipDataset,) = ref_classes("infer_youtube_video_dataset.py", ["InferYoutubeClipDataset"])
    out = {"source": "reference data/youtube_dataset.py + infer_youtube_video_dataset.py classes (ast-extracted, "
                     "unmodified) run on tests/corpus_util.py's corpus", "hw": HW}
    with tempfile.TemporaryDirectory() as root:
        img_dir, data_file, vid_file, subs, ts, vocab = cu.write_corpus(root, hw=HW)
        tok = cu.tokenizer(vocab)
        tf = train_vision_preprocess()

        clip = []
        ds = YoutubeClipDataset(img_dir, data_file, vid_file, tok, 16, 24, transform=tf)
        for seed in (1, 2, 3, 4):
            for i in range(len(ds)):
                seeded(seed)
                img, ids, mask, label = ds[i]
                clip.append({"seed": seed, "i": i, "label": int(label), "ids": ids.tolist(), "mask": mask.tolist(),
                             "img": cu.tensor_digest(img.numpy()), "img_shape": list(img.shape)})
        out["youtube_clip"] = {"clip_frame_num": 16, "max_text_len": 24, "items": clip}

        win = []
        for mode in ("all", "text"):
            ds = WindowClipDataset(img_dir, data_file, vid_file, tok, 8, 24, window_size=2, mode=mode, transform=tf)
            for seed in (1, 2, 3, 5, 8):
                for i in range(len(ds)):
                    seeded(seed + i)
                    img, ids, mask, label, info = ds[i]
                    win.append({"mode": mode, "seed": seed + i, "i": i, "label": int(label), "ids": ids.tolist(),
                                "mask": mask.tolist(), "img": cu.tensor_digest(img.numpy()),
                                "img_shape": list(img.shape),
                                "info": {k: v.tolist() for k, v in info.items()}})
        out["window_clip"] = {"clip_frame_num": 8, "max_text_len": 24, "window_size": 2, "items": win}

        paths = cu.write_clip_jsons(root, img_dir, subs, ts, 16)
        inf = []
        ds = InferYoutubeClipDataset(img_dir, paths, tok, 16, 24, transform=tf)
        for i in range(len(ds)):
            seeded(i)
            img, ids, mask, label = ds[i]
            inf.append({"i": i, "label": int(label), "ids": ids.tolist(), "mask": mask.tolist(),
                        "img": cu.tensor_digest(img.numpy()), "img_shape": list(img.shape)})
        out["infer_clip"] = {"clip_frame_num": 16, "max_text_len": 24, "n": len(ds), "items": inf}

    path = os.path.join(REPO, "tests", "golden", "datasets.json")
    with open(path, "w") as f:
        json.dump(out, f)
    print("wrote", path, {k: len(v["items"]) for k, v in out.items() if isinstance(v, dict)})


if __name__ == "__main__":
    main()
