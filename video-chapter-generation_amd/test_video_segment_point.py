"""Score every clip window of the test videos and report mAP / recall / precision / F — the
reference's `test_video_segment_point.py`, on the MI355X engines.

This mirrors the reference driver:
- BN runs with batch statistics. The driver drops the running stats as at `:116-122`: it sets
  track_running_stats False and running_mean / running_var to None on every BatchNorm2d.
- Windows are scored in clip order with `pred_label = argmax(logits)` and
  `pred_score = prob[:, 1]` (`:185-206`).
- Metrics come from `eval_utils.video_metrics.evaluate_videos`, which restates `:214-377`. It keeps
  the per-video grouping, the seeded random baseline and the final "add last vid" step.

Inputs: `--img_dir` + `--test_clips_json` (and `--test_easy_clips_json` / `--test_hard_clips_json` for
`--data_type easy|hard`, `:150-156`) read the reference's on-disk clip JSON and JPEG frames (u8 frames normalised on
the GPU in "all" mode). Without them (no network here) the clips come from `data.synthetic_dataset`.
"""
import argparse
import json
import os
import random
import sys

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
if _HERE not in sys.path:
    sys.path.insert(0, _HERE)


def drop_bn_running_stats(model):
    n = 0
    for m in model.modules():
        if isinstance(m, torch.nn.BatchNorm2d):
            m.track_running_stats = False
            m.running_mean = None
            m.running_var = None
            n += 1
    return n


@torch.no_grad()
def score_clips(model, dataset, batch_size, device, data_mode="all", num_workers=0):
    from vcg_hip.ingest import is_u8_clips, stage_clips_u8
    loader = torch.utils.data.DataLoader(dataset, shuffle=False, batch_size=batch_size, num_workers=num_workers)
    labels, scores = [], []
    for img_clip, text_ids, attention_mask, _ in loader:
        text_ids, attention_mask = text_ids.to(device), attention_mask.to(device)
        if data_mode == "all" and is_u8_clips(img_clip):  # decoded u8 frames, normalised on the GPU
            staged = stage_clips_u8(img_clip, device, model.compute_dtype())
            logits, prob = model.forward_staged(staged, text_ids, attention_mask)
        elif data_mode == "text":
            logits, prob = model(text_ids, attention_mask)
        elif data_mode == "image":
            logits, prob = model(img_clip.float().to(device))
        elif data_mode == "all":
            logits, prob = model(img_clip.float().to(device), text_ids, attention_mask)
        else:
            raise RuntimeError(f"Unknown data mode {data_mode}")
        labels += logits.float().topk(1, 1, True, True)[1].squeeze(1).cpu().tolist()
        scores += prob[:, 1].float().cpu().tolist()
    for i, info in enumerate(dataset.all_clip_infos):
        info["pred_score"] = scores[i]
        info["pred_label"] = labels[i]
    return dataset.all_clip_infos


def build_parser():
    p = argparse.ArgumentParser(description="video chapter model test (MI355X)")
    p.add_argument("--gpu", default=0, type=int)
    p.add_argument("--data_mode", default="all", type=str)
    p.add_argument("--clip_frame_num", default=16, type=int)
    p.add_argument("--batch_size", default=16, type=int,
                   help="the reference's default (:41): with batch-statistics BN it decides every score")
    p.add_argument("--head_type", default="mlp", type=str)
    p.add_argument("--model_type", default="r50tsm", type=str)
    p.add_argument("--data_type", default="all", type=str, help="all, easy or hard: which clip JSON (:150-156)")
    p.add_argument("--max_text_len", default=100, type=int)
    p.add_argument("--resolution", default=224, type=int)
    p.add_argument("--videos", default=2, type=int, help="synthetic corpus size (no --img_dir)")
    p.add_argument("--precision", default="bf16", choices=["bf16", "fp32"])
    p.add_argument("--ckpt_path", default=None, help="checkpoint written by train_video_segment_point.py")
    # the reference's on-disk inputs (hard-coded at :56-66): frames <img_dir>/<vid>/%05d.jpg named by the clip
    # JSON records' image_paths, one clip JSON per --data_type
    p.add_argument("--img_dir", default=None)
    p.add_argument("--test_clips_json", default=None)
    p.add_argument("--test_easy_clips_json", default=None)
    p.add_argument("--test_hard_clips_json", default=None)
    p.add_argument("--vocab_file", default=None, help="BERT WordPiece vocab.txt (bert-base-uncased's)")
    p.add_argument("--num_workers", default=0, type=int)
    p.add_argument("--clips_json", default=None, help="synthetic corpus: a clip JSON it can rebuild")
    p.add_argument("--result_file", default=None)
    p.add_argument("--seed", default=123, type=int)
    return p


def main(argv=None):
    args = build_parser().parse_args(argv)

    from common_utils import set_random_seed
    from eval_utils.video_metrics import evaluate_videos
    from train_video_segment_point import make_tokenizer, vision_transform
    from vcg_hip.build import build_model

    set_random_seed.use_fix_random_seed(args.seed)
    device = torch.device("cuda", args.gpu)
    torch.cuda.set_device(device)
    model = build_model(args.data_mode, clip_frame_num=args.clip_frame_num, head_type=args.head_type,
                        model_type=args.model_type, seed=args.seed, device=device, precision=args.precision)
    if args.ckpt_path:
        ck = torch.load(args.ckpt_path, map_location=device, weights_only=True)
        model.load_state_dict(ck["model_state_dict"])
    model.eval()
    drop_bn_running_stats(model)
    tok = make_tokenizer(args.vocab_file)
    if args.img_dir:
        from data.infer_youtube_video_dataset import InferYoutubeClipDataset
        jsons = {"all": args.test_clips_json, "easy": args.test_easy_clips_json, "hard": args.test_hard_clips_json}
        if args.data_type not in jsons:
            raise RuntimeError(f"Unknown data_type {args.data_type}")
        if not jsons[args.data_type]:
            raise RuntimeError(f"--data_type {args.data_type} needs --test_{'' if args.data_type == 'all' else args.data_type + '_'}clips_json")
        u8 = args.data_mode == "all"
        ds = InferYoutubeClipDataset(args.img_dir, jsons[args.data_type], tok, args.clip_frame_num, args.max_text_len,
                                     mode=args.data_mode, transform=None if u8 else vision_transform(False), u8=u8)
    else:
        from data.synthetic_dataset import InferYoutubeClipDataset, SyntheticVideoCorpus
        if args.data_type != "all":
            raise RuntimeError("--data_type easy / hard needs the on-disk clip JSONs (--img_dir)")
        corpus = SyntheticVideoCorpus(args.videos, H=args.resolution, W=args.resolution, seed=args.seed + 1)
        ds = InferYoutubeClipDataset(corpus, tok, args.clip_frame_num, args.max_text_len, mode=args.data_mode,
                                     json_path=args.clips_json)
    infos = score_clips(model, ds, args.batch_size, device, args.data_mode, args.num_workers)
    res, vid2cut = evaluate_videos(infos, args.clip_frame_num, getattr(ds, "max_offset", 2), random.Random(args.seed))
    print(json.dumps(res))
    if args.result_file:
        os.makedirs(os.path.dirname(os.path.abspath(args.result_file)), exist_ok=True)
        with open(args.result_file, "w") as f:
            json.dump({"results": res, "vid2cut_points": vid2cut}, f)
    return res


if __name__ == "__main__":
    main()
