"""Export per-clip vision embeddings (`convert2vision_emb.py:131-216`).

The model runs in eval mode with `return_emb=True` over every clip record. For each clip it writes
`<save_dir>/<vid>/vision_emb_<start>_<end>.npy`: a float32 `[T, 2048]` array, the TSM-ResNet
feature of each frame, in the same file layout as the reference. The later stages
(`youtube_chapter_title_dataset.py:223-247`) read these files, and `load_vision_emb` here is that
reader.
"""
import argparse
import os
import sys

import numpy as np
import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
if _HERE not in sys.path:
    sys.path.insert(0, _HERE)


def emb_path(save_dir, vid, start, end):
    return os.path.join(save_dir, vid, f"vision_emb_{start}_{end}.npy")


def load_vision_emb(save_dir, vid, start, end):
    return np.load(emb_path(save_dir, vid, start, end), allow_pickle=False)


@torch.no_grad()
def export_vision_embs(model, dataset, save_dir, batch_size, device):
    loader = torch.utils.data.DataLoader(dataset, shuffle=False, batch_size=batch_size, num_workers=0)
    k = 0
    for img, ids, mask, _ in loader:
        _, _, vision_emb, _ = model(img.float().to(device), ids.to(device), mask.to(device), return_emb=True)
        emb = vision_emb.float().cpu().numpy()
        for i in range(emb.shape[0]):
            info = dataset.all_clip_infos[k + i]
            s, e = info["clip_start_end"]
            path = emb_path(save_dir, info["vid"], s, e)
            os.makedirs(os.path.dirname(path), exist_ok=True)
            np.save(path, emb[i].astype(np.float32))
        k += emb.shape[0]
    return k


def main(argv=None):
    p = argparse.ArgumentParser(description="export vision embeddings (MI355X)")
    p.add_argument("--gpu", default=0, type=int)
    p.add_argument("--clip_frame_num", default=16, type=int)
    p.add_argument("--batch_size", default=32, type=int)
    p.add_argument("--max_text_len", default=100, type=int)
    p.add_argument("--resolution", default=224, type=int)
    p.add_argument("--videos", default=2, type=int)
    p.add_argument("--precision", default="bf16", choices=["bf16", "fp32"])
    p.add_argument("--ckpt_path", default=None)
    p.add_argument("--clips_json", default=None)
    p.add_argument("--save_dir", default="./vision_emb")
    p.add_argument("--seed", default=123, type=int)
    args = p.parse_args(argv)

    from data.synthetic_dataset import HashTokenizer, InferYoutubeClipDataset, SyntheticVideoCorpus
    from vcg_hip.build import build_two_stream

    device = torch.device("cuda", args.gpu)
    torch.cuda.set_device(device)
    model = build_two_stream(clip_frame_num=args.clip_frame_num, seed=args.seed, device=device,
                             precision=args.precision)
    if args.ckpt_path:
        model.load_state_dict(torch.load(args.ckpt_path, map_location=device, weights_only=True)["model_state_dict"])
    model.eval()
    corpus = SyntheticVideoCorpus(args.videos, H=args.resolution, W=args.resolution, seed=args.seed + 1)
    ds = InferYoutubeClipDataset(corpus, HashTokenizer(), args.clip_frame_num, args.max_text_len,
                                 json_path=args.clips_json)
    n = export_vision_embs(model, ds, args.save_dir, args.batch_size, device)
    print(f"wrote {n} clip embeddings under {args.save_dir}")
    return n


if __name__ == "__main__":
    main()
