"""Data-parallel training of the clip scorer: one process per GPU, RCCL all-reduce over xGMI.

This replaces the reference's `train_video_segment_ddp.py`. The reference wraps the model in
`DDP(model)` with NCCL and 25 MB buckets, all-reducing on every backward (`:131-148`); it draws
data with a DistributedSampler (`:210-243`), broadcasts the rank-0 parameters (`:261-263`) and
averages the validation metric with `all_gather_object` (`:276-281`). Here:
- `vcg_hip.ddp.GradAllReducer` reduces the flat fp32 gradient buffer in 25 MB contiguous
  buckets (DDP's default). Each bucket is sent as an async RCCL all_reduce(SUM) as soon as the native backward
  reports its parameters final, so the exchange overlaps the rest of the backward.
- The 1/world average is folded into the fused AdamW (`grad_scale`).
- Gradient accumulation reduces only on the last micro-step (`reducer.enabled`). The sum of the
  micro-step gradients is linear, so the result equals DDP's reduce-every-backward.
- Parameters start identical through one broadcast of the flat parameter buffer; the BatchNorm running
  statistics are re-broadcast from rank 0 before every training forward (DDP's broadcast_buffers=True),
  as one collective over a flat buffer (`vcg_hip.ddp.BufferBroadcaster`).

Launch: `python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 train_video_segment_ddp.py`.
"""
import argparse
import glob
import os
import re
import sys

import torch
import torch.distributed as dist

_HERE = os.path.dirname(os.path.abspath(__file__))
if _HERE not in sys.path:
    sys.path.insert(0, _HERE)

from train_video_segment_point import TrainerConfig, lr_multiplier  # noqa: E402


CKPT_RE = re.compile(r"_(\d+)(?:_score_[\d.]+)?\.pth$")


def find_latest_checkpoint(ckpt_path, rank=0):
    """(path, epoch) of the newest checkpoint, found on rank 0 and broadcast (`train_video_segment_ddp.py:176-207`);
    (None, 0) when there is none. The epoch rule is the reference's `_(\\d+)(?:_score_[\\d.]+)?\\.pth$` (re.search).
    A directory ckpt_path ("DIR/", or an existing directory) is searched exactly as the reference does: every
    DIR/*.pth whose name matches, whatever its prefix. A name prefix ("DIR/run", "DIR/run.pth") -- where the
    reference's directory glob finds nothing and so never resumes -- is searched where checkpoint_path() writes:
    DIR/run_<epoch>[_score_<s>].pth only."""
    info = (None, 0)
    if rank == 0 and ckpt_path:
        if ckpt_path.endswith(os.sep) or os.path.isdir(ckpt_path):
            folder, name_re, match = ckpt_path, CKPT_RE, CKPT_RE.search
        else:
            base = os.path.splitext(ckpt_path)[0]
            folder, prefix = os.path.dirname(base) or ".", os.path.basename(base)
            match = re.compile(re.escape(prefix) + CKPT_RE.pattern).fullmatch
        best = (None, -1)
        for f in sorted(glob.glob(os.path.join(glob.escape(folder), "*.pth"))):
            m = match(os.path.basename(f))
            if m and int(m.group(1)) > best[1]:
                best = (f, int(m.group(1)))
        if best[0] is not None:
            info = best
    if dist.is_initialized():
        obj = [info]
        dist.broadcast_object_list(obj, src=0)
        info = obj[0]
    return info


def checkpoint_path(ckpt_path, epoch, best_result, is_best):
    """`train_video_segment_ddp.py:150-173`'s names: <base>_<epoch>_score_<best:.4f>.pth or <base>_<epoch>.pth."""
    base = os.path.splitext(ckpt_path)[0]
    return f"{base}_{epoch}_score_{best_result:.4f}.pth" if is_best else f"{base}_{epoch}.pth"


class DDPTrainer:
    def __init__(self, model, train_dataset, test_dataset, config, rank, world_size, device):
        from vcg_hip.ddp import BufferBroadcaster, GradAllReducer, broadcast_parameters
        self.model, self.train_dataset, self.test_dataset = model, train_dataset, test_dataset
        self.config, self.rank, self.world, self.device = config, rank, world_size, device
        self.optimizer = model.configure_optimizers(config)
        self.optimizer.grad_scale = 1.0 / world_size
        broadcast_parameters(model)
        self.reducer = GradAllReducer(model.native_flat())
        # both models report their gradients final block by block (buckets overlap the backward); whatever no hook
        # reported (the window model's heads) is reduced by finish()
        self.overlap = hasattr(model, "set_grad_hooks")
        if self.overlap:
            model.set_grad_hooks(self.reducer)
        # DDP(model)'s broadcast_buffers=True: rank 0's BatchNorm running stats before every training forward
        self.buffers = BufferBroadcaster(model)
        self.history = []
        self.start_epoch, self.best_result = 0, float("-inf")

    def resume(self):
        """Continue from the newest checkpoint under config.ckpt_path (`:176-207,245-263`): rank 0 finds it and
        broadcasts its name; every rank loads the model and optimizer state from it (the reference loads the
        optimizer state on rank 0 only, leaving the other ranks' Adam moments at zero), then rank 0's parameters are
        broadcast as at start."""
        from vcg_hip.ddp import broadcast_parameters
        path, _ = find_latest_checkpoint(self.config.ckpt_path, self.rank)
        if path is None:
            return None
        ck = torch.load(path, map_location=self.device, weights_only=True)
        self.model.load_state_dict(ck["model_state_dict"])
        self.optimizer.load_state_dict(ck["optimizer_state_dict"])
        self.start_epoch, self.best_result = int(ck["epoch"]), float(ck["best_result"])
        broadcast_parameters(self.model)
        return path

    def save_checkpoint(self, epoch, best_result, is_best=False):
        """Rank 0 writes the reference's checkpoint dict (`:150-173`)."""
        if self.rank != 0 or self.config.ckpt_path is None:
            return None
        path = checkpoint_path(self.config.ckpt_path, epoch, best_result, is_best)
        os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
        torch.save({"epoch": epoch, "best_result": best_result, "model_state_dict": self.model.state_dict(),
                    "optimizer_state_dict": self.optimizer.state_dict()}, path)
        return path

    def fit(self, val_every=30, save_every=10, save_on_val_epochs=False):
        """The reference's epoch loop (`:265-290`): validation every `val_every` epochs (rank-averaged metric; a best
        checkpoint when it improves), else a regular checkpoint every `save_every` epochs (the reference's `elif`: a
        validation epoch never writes a regular checkpoint). save_on_val_epochs (not the reference's cadence): a
        validation epoch that wrote no best checkpoint (NaN or no improvement) takes the regular save too."""
        best, result = self.best_result, None
        for epoch in range(self.start_epoch + 1, self.config.max_epochs + 1):
            self.run_epoch("train", epoch)
            if self.test_dataset is not None and epoch % val_every == 0:
                result = self.run_epoch("infer_test", epoch)
                if self.rank == 0:
                    print(f"epoch {epoch}: val {result}")
                if result == result and result > best:
                    best = result
                    self.save_checkpoint(epoch, best, is_best=True)
                elif save_on_val_epochs and epoch % save_every == 0:
                    self.save_checkpoint(epoch, best, is_best=False)
            elif epoch % save_every == 0:
                self.save_checkpoint(epoch, best, is_best=False)
        self.best_result = best
        return result

    def run_epoch(self, split, epoch):
        from vcg_hip.ddp import all_gather_object
        from vcg_hip.functions import cross_entropy
        from eval_utils.video_metrics import trainer_video_auc_map
        is_train = split == "train"
        ds = self.train_dataset if is_train else self.test_dataset
        self.model.train(is_train)
        sampler = torch.utils.data.distributed.DistributedSampler(ds, num_replicas=self.world, rank=self.rank,
                                                                  shuffle=is_train)
        sampler.set_epoch(epoch)
        bs = self.config.batch_size if is_train else self.config.val_batch_size
        loader = torch.utils.data.DataLoader(ds, batch_size=bs, sampler=sampler, num_workers=self.config.num_workers)
        accum = self.config.gradient_accumulation_steps
        scored = []
        order = list(sampler)
        window = []
        for it, batch in enumerate(loader):
            img, ids, mask, label = (batch[0].float().to(self.device), batch[1].to(self.device),
                                     batch[2].to(self.device), batch[3].to(self.device))
            clip_info = batch[4] if len(batch) > 4 else None  # the window model's window metadata
            last_micro = (it + 1) % accum == 0
            self.reducer.enabled = is_train and self.world > 1 and last_micro
            if is_train and self.world > 1:
                self.buffers()
            with torch.set_grad_enabled(is_train):
                logits, prob = (self.model(img, ids, mask, clip_info) if clip_info is not None
                                else self.model(img, ids, mask))
                loss = cross_entropy(logits, label)
            if not is_train and clip_info is not None:
                window += list(zip(label.cpu().tolist(), prob[:, 1].float().cpu().tolist()))
                continue
            if not is_train:
                idx = order[it * bs:it * bs + len(label)]
                for k, s in zip(idx, prob[:, 1].float().cpu().tolist()):
                    scored.append((k, s))
                continue
            (loss / accum).backward()
            if last_micro:
                if self.overlap:
                    self.reducer.finish()
                else:
                    self.reducer.reduce_all()
                self.optimizer.clip_and_step(self.config.grad_norm_clip)
                self.model.zero_grad()
                if self.config.lr_decay:
                    for g in self.optimizer.param_groups:
                        g["lr"] = self.config.learning_rate * lr_multiplier(self.config, epoch)
                self.history.append({"epoch": epoch, "it": it, "loss": loss.item()})
        self.reducer.enabled = self.world > 1
        if is_train:
            return None
        if window:  # window model: average precision of the target clips over every rank's windows
            from sklearn.metrics import average_precision_score
            allw = [x for part in all_gather_object(window) for x in part]
            labels = [a for a, _ in allw]
            return float(average_precision_score(labels, [b for _, b in allw])) if 0 < sum(labels) < len(labels) \
                else float("nan")
        for part in all_gather_object(scored):  # every rank gets every clip's score (clip order restored)
            for k, s in part:
                ds.all_clip_infos[k]["pred_score"] = s
        return trainer_video_auc_map(ds.all_clip_infos)[1]


def main(argv=None):
    p = argparse.ArgumentParser(description="video chapter model, data parallel (MI355X, RCCL)")
    p.add_argument("--epoch", default=2, type=int)
    p.add_argument("--batch_size", default=4, type=int)
    p.add_argument("--clip_frame_num", default=16, type=int)
    p.add_argument("--max_text_len", default=100, type=int)
    p.add_argument("--resolution", default=224, type=int)
    p.add_argument("--videos", default=16, type=int)
    p.add_argument("--precision", default="bf16", choices=["bf16", "fp32"])
    p.add_argument("--seed", default=123, type=int)
    p.add_argument("--window_size", default=0, type=int,
                   help="0: the point clip scorer; w > 0: the window model of the reference's DDP driver "
                        "(two_stream_window.TwoStream over 2w+1 clips, WindowClipDataset)")
    p.add_argument("--head_type", default="cross_attn", help="window model head (reference default cross_attn)")
    p.add_argument("--data_dir", default=None, help="window model: directory for the reference-format corpus")
    p.add_argument("--ckpt_path", default=None,
                   help="checkpoint directory (+ name prefix); training resumes from its newest checkpoint")
    p.add_argument("--val_every", default=1, type=int, help="validate every N epochs (the reference: 30)")
    p.add_argument("--save_every", default=10, type=int, help="regular checkpoint every N epochs (the reference: 10)")
    p.add_argument("--save_on_val_epochs", action="store_true",
                   help="also take the regular checkpoint on validation epochs without a new best (not the reference)")
    args = p.parse_args(argv)

    from common_utils import set_random_seed
    from data.synthetic_dataset import HashTokenizer, InferYoutubeClipDataset, SyntheticVideoCorpus, YoutubeClipDataset
    from vcg_hip.build import build_two_stream

    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0))
    device = torch.device("cuda", local)
    torch.cuda.set_device(device)
    if world > 1:
        dist.init_process_group("nccl", device_id=device)
    set_random_seed.use_fix_random_seed(args.seed + rank)
    tok = HashTokenizer()
    if args.window_size > 0:
        return _window_main(args, rank, world, device, tok)
    train_ds = YoutubeClipDataset(SyntheticVideoCorpus(args.videos, H=args.resolution, W=args.resolution, seed=args.seed),
                                  tok, args.clip_frame_num, args.max_text_len)
    test_ds = InferYoutubeClipDataset(SyntheticVideoCorpus(2, H=args.resolution, W=args.resolution, seed=args.seed + 1),
                                      tok, args.clip_frame_num, args.max_text_len)
    model = build_two_stream(clip_frame_num=args.clip_frame_num, seed=args.seed, device=device, precision=args.precision)
    conf = TrainerConfig(max_epochs=args.epoch, batch_size=args.batch_size, val_batch_size=args.batch_size * 8,
                         gradient_accumulation_steps=4, num_workers=0, lr_decay=True,
                         warmup_epochs=args.epoch // 100, final_epochs=args.epoch // 100 * 90, ckpt_path=args.ckpt_path)
    return _fit(DDPTrainer(model, train_ds, test_ds, conf, rank, world, device), args, world)


def _fit(tr, args, world):
    resumed = tr.resume()
    if resumed and tr.rank == 0:
        print(f"resumed from {resumed} (epoch {tr.start_epoch}, best {tr.best_result})")
    result = tr.fit(args.val_every, args.save_every, args.save_on_val_epochs)
    if world > 1:
        dist.destroy_process_group()
    return result


def _window_main(args, rank, world, device, tok):
    """The reference driver's own configuration (train_video_segment_ddp.py:445-564): the window TwoStream with
    WindowClipDataset batches over a corpus in the reference's on-disk format (written from the synthetic corpus)."""
    import tempfile

    from data.synthetic_dataset import SyntheticVideoCorpus
    from data.transforms import test_vision_preprocess, train_vision_preprocess
    from data.youtube_dataset import WindowClipDataset
    from vcg_hip.build import build_window_two_stream
    root = args.data_dir or tempfile.mkdtemp(prefix="vcg_win_")
    paths = {}
    for split, n, seed in (("train", args.videos, args.seed), ("test", 2, args.seed + 1)):
        d = os.path.join(root, split)
        if rank == 0 and not os.path.exists(os.path.join(d, f"{split}.txt")):
            SyntheticVideoCorpus(n, H=args.resolution, W=args.resolution, seed=seed).write(d, f"{split}.txt")
        paths[split] = (os.path.join(d, "frames"), os.path.join(d, "subtitles", "data.csv"), os.path.join(d, f"{split}.txt"))
    if world > 1:
        dist.barrier()
    train_ds = WindowClipDataset(*paths["train"], tok, args.clip_frame_num, args.max_text_len, args.window_size,
                                 transform=train_vision_preprocess())
    test_ds = WindowClipDataset(*paths["test"], tok, args.clip_frame_num, args.max_text_len, args.window_size,
                                transform=test_vision_preprocess())
    model = build_window_two_stream(clip_frame_num=args.clip_frame_num, window_size=args.window_size,
                                    head_type=args.head_type, seed=args.seed, device=device, precision=args.precision)
    conf = TrainerConfig(max_epochs=args.epoch, batch_size=args.batch_size, val_batch_size=args.batch_size,
                         gradient_accumulation_steps=4, num_workers=0, lr_decay=True,
                         warmup_epochs=args.epoch // 100, final_epochs=args.epoch // 100 * 90, ckpt_path=args.ckpt_path)
    return _fit(DDPTrainer(model, train_ds, test_ds, conf, rank, world, device), args, world)


if __name__ == "__main__":
    main()
