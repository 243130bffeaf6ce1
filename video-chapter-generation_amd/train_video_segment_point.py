"""Train the clip scorer: the reference's `train_video_segment_point.py`, with the MI355X engines
underneath.

`TrainerConfig` / `Trainer` keep the reference's names, fields and call protocol
(`train_video_segment_point.py:31-279`). That covers `Trainer(model, train_dataset, test_dataset,
config)`, `.device` set by attribute, `.train()`, and `.run_epoch(split, epoch, dataset)`, which
returns the validation mAP. The step arithmetic is also the same:
- loss / accumulation steps, backward every iteration;
- every `gradient_accumulation_steps` iterations: clip to `grad_norm_clip`, AdamW, zero_grad;
- LR warm-up `max(epoch / warmup, 0.01)`, then cosine `max(0.001, 0.5 (1 + cos(pi p)))` or the
  "exp" staircase (`:205-233`).

Differences:
- Clip + AdamW is one fused device pass (`FusedAdamW.clip_and_step`).
- Inputs may already be GPU tensors.
- `--img_dir/--data_file/--vid_file/--test_clips_json` read the reference's on-disk corpus (JPEG frames, CSV,
  subtitle JSON, clip JSON); in "all" mode the frames stay u8 until the GPU normalises them (vcg_hip/ingest.py).
  Without them (no network here) `__main__` trains on `data.synthetic_dataset`.
- Checkpoints are plain tensors (`torch.save` of state dicts), so they load with `weights_only=True`.
"""
import argparse
import logging
import math
import os
import sys

import numpy as np
import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
if _HERE not in sys.path:
    sys.path.insert(0, _HERE)

from eval_utils.video_metrics import trainer_video_auc_map  # noqa: E402
from vcg_hip.functions import cross_entropy  # noqa: E402
from vcg_hip.ingest import is_u8_clips, stage_clips_u8  # noqa: E402

logger = logging.getLogger(__name__)


class TrainerConfig:
    data_mode = "all"
    max_epochs = 3000
    start_epoch = 0
    best_result = float("-inf")
    block_size = 50
    batch_size = 8
    learning_rate = 1e-5
    betas = (0.9, 0.95)
    grad_norm_clip = 1.0
    weight_decay = 0.01
    lr_decay = False
    lr_decay_type = "cosine"
    warmup_epochs = 200
    final_epochs = 2500
    ckpt_path = None
    num_workers = 8
    tensorboard_writer = None
    gradient_accumulation_steps = 4

    def __init__(self, **kwargs):
        for k, v in kwargs.items():
            setattr(self, k, v)


def lr_multiplier(config, epoch):
    """LR multiplier of `train_video_segment_point.py:205-233` (applied after each optimiser step)."""
    if epoch < config.warmup_epochs:
        return max(epoch / config.warmup_epochs, 1e-2)
    progress = epoch / config.final_epochs if epoch < config.final_epochs else 1.0
    if config.lr_decay_type == "cosine":
        return max(0.001, 0.5 * (1.0 + math.cos(math.pi * progress)))
    if config.lr_decay_type == "exp":
        th = 1 / 5
        if progress < th:
            return 1
        if th < progress < th * 2:
            return 0.1
        if th * 2 < progress < th * 3:
            return 0.01
        return 0.001
    raise RuntimeError("Unknown learning rate decay type")


def _binary_auc_map(labels, scores):
    from sklearn import metrics
    pos = labels.count(1)
    if len(labels) > pos > 0:
        fpr, tpr, _ = metrics.roc_curve(labels, scores, pos_label=1)
        return metrics.auc(fpr, tpr), metrics.average_precision_score(labels, scores)
    return 0, 0


class Trainer:
    def __init__(self, model, train_dataset, test_dataset, config):
        self.model = model
        self.train_dataset = train_dataset
        self.test_dataset = test_dataset
        self.config = config
        self.device = "cuda"
        self.optimizer = None
        self.history = []

    def save_checkpoint(self, epoch, best_result, is_best=True):
        raw = self.model.module if hasattr(self.model, "module") else self.model
        base = os.path.splitext(self.config.ckpt_path)[0]
        os.makedirs(os.path.dirname(os.path.abspath(self.config.ckpt_path)), exist_ok=True)
        path = f"{base}_{epoch}_score_{best_result:.4f}.pth" if is_best else f"{base}_{epoch}.pth"
        torch.save({"epoch": epoch, "best_result": best_result, "model_state_dict": raw.state_dict(),
                    "optimizer_state_dict": self.optimizer.state_dict()}, path)
        return path

    def train(self):
        raw = self.model.module if hasattr(self.model, "module") else self.model
        self.optimizer = raw.configure_optimizers(self.config)
        best = self.config.best_result
        for epoch in range(self.config.start_epoch + 1, self.config.max_epochs + 1):
            self.run_epoch("train", epoch, self.train_dataset)
            if self.test_dataset is not None and (epoch % 30 == 0 or epoch in (1, 15, 45)):
                result = self.run_epoch("infer_test", epoch, self.test_dataset)
                if result > best:
                    best = result
                    if self.config.ckpt_path is not None:
                        self.save_checkpoint(epoch, best, is_best=True)
        return best

    def _forward(self, img_clip, text_ids, attention_mask):
        mode = self.config.data_mode
        if mode == "all" and is_u8_clips(img_clip):
            # decoded u8 frames (data.* datasets with u8=True): uploaded as bytes, normalised on the GPU into the
            # stem's layout (vcg_hip/ingest.py), the same ToTensor + Normalize map as the f32 transform
            raw = self.model.module if hasattr(self.model, "module") else self.model
            staged = stage_clips_u8(img_clip, text_ids.device, raw.compute_dtype())
            return self.model.forward_staged(staged, text_ids, attention_mask)
        if mode == "text":
            return self.model(text_ids, attention_mask)
        if mode == "image":
            return self.model(img_clip)
        if mode == "all":
            return self.model(img_clip, text_ids, attention_mask)
        raise RuntimeError(f"Unknown data mode {mode}")

    def run_epoch(self, split, epoch, dataset):
        is_train = split == "train"
        self.model.train(is_train)
        bs = self.config.batch_size if is_train else self.config.batch_size * 8
        loader = torch.utils.data.DataLoader(dataset, shuffle=is_train, batch_size=bs,
                                             num_workers=self.config.num_workers)
        losses = []
        accum = self.config.gradient_accumulation_steps
        for it, (img_clip, text_ids, attention_mask, label) in enumerate(loader):
            if torch.is_tensor(img_clip) and not is_u8_clips(img_clip):
                img_clip = img_clip.float().to(self.device)
            text_ids = text_ids.to(self.device)
            attention_mask = attention_mask.to(self.device)
            label = label.to(self.device)
            with torch.set_grad_enabled(is_train):
                logits, prob = self._forward(img_clip, text_ids, attention_mask)
                loss = cross_entropy(logits, label)  # native vcg_cross_entropy (mean CE, :165)
            scores = prob[:, 1].detach().float().cpu().numpy()
            if not is_train:
                start = it * bs
                for i in range(start, start + len(scores)):
                    dataset.all_clip_infos[i]["pred_score"] = float(scores[i - start])
                losses.append(loss.item())
                continue
            auc, m_ap = _binary_auc_map(label.cpu().tolist(), scores)
            (loss / accum).backward()
            if (it + 1) % accum == 0:
                self.optimizer.clip_and_step(self.config.grad_norm_clip)
                self.model.zero_grad()
                lr = self.config.learning_rate
                if self.config.lr_decay:
                    lr = self.config.learning_rate * lr_multiplier(self.config, epoch)
                    for g in self.optimizer.param_groups:
                        g["lr"] = lr
                self.history.append({"epoch": epoch, "it": it, "loss": loss.item(), "auc": auc, "m_ap": m_ap,
                                     "lr": lr})
                w = self.config.tensorboard_writer
                if w is not None:  # the reference's scalars (:244-248); loss is the un-divided CE
                    n_iter = epoch * len(loader) + it
                    w.add_scalar("Train/loss", loss.item(), n_iter)
                    if auc:
                        w.add_scalar("Train/auc", auc, n_iter)
                        w.add_scalar("Train/m_ap", m_ap, n_iter)
        if not is_train:
            test_auc, test_map = trainer_video_auc_map(dataset.all_clip_infos)
            test_loss = float(np.mean(losses))
            print(f"{split}, loss: {test_loss}, auc {test_auc}, m_ap {test_map}")
            w = self.config.tensorboard_writer
            if w is not None:  # (:279-281)
                w.add_scalar(f"{split}/loss", test_loss, epoch)
                w.add_scalar(f"{split}/auc", test_auc, epoch)
                w.add_scalar(f"{split}/m_ap", test_map, epoch)
            return test_map
        return None


def build_model(args, device):
    from vcg_hip.build import build_model as _build
    return _build(args.data_mode, clip_frame_num=args.clip_frame_num, hidden_size=128, head_type=args.head_type,
                  model_type=args.model_type, seed=args.seed, device=device, precision=args.precision)


def make_tokenizer(vocab_file):
    """BertTokenizer over a local WordPiece vocab (the reference loads 'bert-base-uncased' from the hub,
    `train_video_segment_point.py:324`; there is no network here), else the synthetic corpus's tokenizer."""
    if vocab_file:
        from transformers import BertTokenizer
        return BertTokenizer(vocab_file=vocab_file, do_lower_case=True)
    from data.synthetic_dataset import HashTokenizer
    return HashTokenizer()


def vision_transform(train):
    """`train_video_segment_point.py:377-386` (data/transforms.py restates the torchvision classes)."""
    from data import transforms as T
    norm = [T.ToTensor(), T.Normalize(mean=T.IMAGENET_MEAN, std=T.IMAGENET_STD)]
    return T.Compose(([T.RandomApply([T.ColorJitter()], p=0.5)] if train else []) + norm)


def disk_datasets(args, tok):
    """The reference's datasets over a corpus on disk (`train_video_segment_point.py:388-389`). In "all" mode the
    frames stay u8 for the GPU ingest (vcg_hip/ingest.py); the other modes use the f32 transforms."""
    from data.infer_youtube_video_dataset import InferYoutubeClipDataset
    from data.youtube_dataset import YoutubeClipDataset
    u8 = args.data_mode == "all"
    train = YoutubeClipDataset(args.img_dir, args.data_file, args.vid_file, tok, args.clip_frame_num,
                               args.max_text_len, mode=args.data_mode, transform=None if u8 else vision_transform(True),
                               subtitle_dir=args.subtitle_dir, u8=u8)
    test = None
    if args.test_clips_json:
        test = InferYoutubeClipDataset(args.img_dir, args.test_clips_json, tok, args.clip_frame_num, args.max_text_len,
                                       mode=args.data_mode, transform=None if u8 else vision_transform(False), u8=u8)
    return train, test


def main(argv=None):
    p = argparse.ArgumentParser(description="video chapter model (MI355X)")
    p.add_argument("--gpu", default=0, type=int)
    p.add_argument("--data_mode", default="all", type=str)
    p.add_argument("--clip_frame_num", default=16, type=int)
    p.add_argument("--epoch", default=300, type=int)
    p.add_argument("--batch_size", default=4, type=int)
    p.add_argument("--lr_decay_type", default="cosine", type=str)
    p.add_argument("--head_type", default="mlp", type=str)
    p.add_argument("--model_type", default="r50tsm", type=str, help="r50tsm or r50 (image mode)")
    p.add_argument("--max_text_len", default=100, type=int)
    p.add_argument("--resolution", default=224, type=int)
    p.add_argument("--videos", default=8, type=int, help="synthetic corpus size (no --img_dir)")
    p.add_argument("--precision", default="bf16", choices=["bf16", "fp32"])
    p.add_argument("--seed", default=123, type=int)
    p.add_argument("--ckpt_path", default=None)
    # the reference's on-disk corpus (its hard-coded paths, :307-318): frames <img_dir>/<vid>/%05d.jpg, the dataset
    # CSV, the split's vid list, subtitles <subtitle_dir>/*/subtitle_<vid>.json, the validation clip JSON
    p.add_argument("--img_dir", default=None)
    p.add_argument("--data_file", default=None)
    p.add_argument("--vid_file", default=None)
    p.add_argument("--subtitle_dir", default=None)
    p.add_argument("--test_clips_json", default=None)
    p.add_argument("--vocab_file", default=None, help="BERT WordPiece vocab.txt (bert-base-uncased's)")
    p.add_argument("--num_workers", default=0, type=int)
    p.add_argument("--tensorboard_log", default=None)
    args = p.parse_args(argv)

    from common_utils import set_random_seed

    set_random_seed.use_fix_random_seed(args.seed)
    device = torch.device("cuda", args.gpu)
    torch.cuda.set_device(device)
    tok = make_tokenizer(args.vocab_file)
    if args.img_dir:
        train_ds, test_ds = disk_datasets(args, tok)
    else:
        from data.synthetic_dataset import InferYoutubeClipDataset, SyntheticVideoCorpus, YoutubeClipDataset
        corpus = SyntheticVideoCorpus(args.videos, H=args.resolution, W=args.resolution, seed=args.seed)
        test_corpus = SyntheticVideoCorpus(max(2, args.videos // 4), H=args.resolution, W=args.resolution,
                                           seed=args.seed + 1)
        train_ds = YoutubeClipDataset(corpus, tok, args.clip_frame_num, args.max_text_len, mode=args.data_mode)
        test_ds = InferYoutubeClipDataset(test_corpus, tok, args.clip_frame_num, args.max_text_len, mode=args.data_mode)
    model = build_model(args, device)
    writer = None
    if args.tensorboard_log:
        from common_utils.scalar_log import summary_writer
        writer = summary_writer(args.tensorboard_log)
    conf = TrainerConfig(data_mode=args.data_mode, max_epochs=args.epoch, batch_size=args.batch_size,
                         gradient_accumulation_steps=4, learning_rate=1e-5, block_size=args.max_text_len,
                         lr_decay_type=args.lr_decay_type, lr_decay=True, warmup_epochs=args.epoch // 100,
                         final_epochs=args.epoch // 100 * 90, num_workers=args.num_workers, ckpt_path=args.ckpt_path,
                         tensorboard_writer=writer)
    trainer = Trainer(model, train_ds, test_ds, conf)
    trainer.device = device
    return trainer.train()


if __name__ == "__main__":
    main()
