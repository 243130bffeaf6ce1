"""The reference-shaped drivers end to end on the GPU at a tiny size (T=4 frames of 64², L=32):
train (Trainer: accumulation, fused clip+AdamW, LR schedule, validation mAP), test (batch-stats BN,
per-video metrics), vision-embedding export (npy files), and the data-parallel driver at world 1."""
import math
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

TINY = ["--clip_frame_num", "4", "--resolution", "64", "--max_text_len", "32"]


def test_train_driver(tmp_path):
    import train_video_segment_point as drv
    from data.synthetic_dataset import HashTokenizer, InferYoutubeClipDataset, SyntheticVideoCorpus, YoutubeClipDataset
    from vcg_hip.build import build_model
    dev = torch.device("cuda", 0)
    tok = HashTokenizer()
    train = YoutubeClipDataset(SyntheticVideoCorpus(8, 30, 50, H=64, W=64, seed=1), tok, 4, 32)
    test = InferYoutubeClipDataset(SyntheticVideoCorpus(2, 30, 50, H=64, W=64, seed=2), tok, 4, 32)
    model = build_model("all", clip_frame_num=4, seed=123, device=dev, precision="bf16")
    conf = drv.TrainerConfig(max_epochs=1, batch_size=2, gradient_accumulation_steps=2, num_workers=0, lr_decay=True,
                             warmup_epochs=0, final_epochs=0, ckpt_path=str(tmp_path / "ck.pth"))
    tr = drv.Trainer(model, train, test, conf)
    tr.device = dev
    best = tr.train()
    assert len(tr.history) == 2 and all(math.isfinite(h["loss"]) for h in tr.history)
    assert tr.history[-1]["lr"] == pytest.approx(1e-5 * 0.001)    # final_epochs 0 -> progress 1 -> floor
    assert all("pred_score" in c for c in test.all_clip_infos)
    if math.isfinite(best):
        assert any(f.name.startswith("ck_1_score") for f in tmp_path.iterdir())
        ck = torch.load(next(tmp_path.iterdir()), weights_only=True)
        assert set(ck) == {"epoch", "best_result", "model_state_dict", "optimizer_state_dict"}


def test_test_driver(tmp_path):
    import test_video_segment_point as drv
    out = tmp_path / "res.json"
    res = drv.main(TINY + ["--videos", "2", "--batch_size", "8", "--result_file", str(out)])
    for k in ("mAP", "recall", "precision@3", "f-score@5_rand"):
        assert k in res
    assert 0.0 <= res["mAP"] <= 1.0
    assert out.exists()


def test_vision_emb_export(tmp_path):
    import convert2vision_emb as drv
    n = drv.main(TINY + ["--videos", "1", "--batch_size", "8", "--save_dir", str(tmp_path)])
    files = sorted(tmp_path.rglob("vision_emb_*.npy"))
    assert len(files) == n > 0
    a = np.load(files[0], allow_pickle=False)
    assert a.shape == (4, 2048) and a.dtype == np.float32 and np.isfinite(a).all()


def test_ddp_driver_world1():
    import train_video_segment_ddp as drv
    os.environ.pop("WORLD_SIZE", None)
    r = drv.main(TINY + ["--epoch", "1", "--batch_size", "2", "--videos", "8"])
    assert r is None or r != r or 0.0 <= r <= 1.0


def test_bench_script_small():
    """bench.py end to end at a tiny size (the contract's JSON line: metric, value, roofline with the per-launch
    accounting), so a broken bench is caught by the GPU suite, not at round end."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--steps", "1", "--warmup", "1", "--batch",
                          "2", "--frames", "4", "--res", "112", "--tokens", "32", "--no-cpu-baseline"],
                         capture_output=True, text=True, timeout=300, cwd=root)
    assert out.returncode == 0, out.stderr[-2000:]
    d = json.loads(out.stdout.strip().splitlines()[-1])
    for k in ("metric", "value", "unit", "n_gpus", "ms_per_step", "roofline", "roofline_step", "config"):
        assert k in d, k
    assert d["value"] > 0 and d["roofline"]["bound"] in ("hbm", "mfma") and 0 < d["roofline"]["frac"] < 1
    assert 0 < d["roofline"]["per_launch_roofline"]["frac"] <= 1


@pytest.mark.parametrize("head_type", ["cross_attn", "self_attn"])
def test_ddp_driver_window_model_world1(tmp_path, head_type):
    """The reference DDP driver's own configuration: the window model (window_size 1, cross_attn head -- and the
    self_attn head at the reference's default dropout) trained from WindowClipDataset batches read from a
    reference-format corpus on disk (JPEG frames, subtitle JSON, CSV)."""
    import train_video_segment_ddp as drv
    os.environ.pop("WORLD_SIZE", None)
    r = drv.main(TINY + ["--epoch", "1", "--batch_size", "2", "--videos", "4", "--window_size", "1",
                         "--head_type", head_type, "--data_dir", str(tmp_path)])
    assert r is None or r != r or 0.0 <= r <= 1.0
    assert (tmp_path / "train" / "subtitles" / "data.csv").exists()
