"""The reference-shaped drivers on a corpus written in the reference's on-disk layout (JPEG frames %05d.jpg, the
dataset CSV, subtitle JSON, the eval clip JSON of flat_video2clip_for_quick_infer.py) with a real
transformers.BertTokenizer over a local vocab: train_video_segment_point.py (`:377-389`),
test_video_segment_point.py (`:148-162`, --data_type), the u8 GPU ingest against the f32 host transform, DDP
checkpoint save / resume (`train_video_segment_ddp.py:176-207,288-290`), and `bench.py --gpus 2` launching its own
two ranks (gloo rehearsal on this one-GPU box)."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TINY = ["--clip_frame_num", "16", "--max_text_len", "32"]


@pytest.fixture(scope="module")
def corpus(tmp_path_factory):
    from corpus_util import VIDS, write_clip_jsons, write_corpus
    root = str(tmp_path_factory.mktemp("corpus"))
    img_dir, data_file, vid_file, subs, timestamps, vocab = write_corpus(root, hw=64)
    jsons = write_clip_jsons(root, img_dir, subs, timestamps, clip_frame_num=16)
    allj = os.path.join(root, "clips_all.json")
    recs = [r for p in jsons for r in json.load(open(p))]
    with open(allj, "w") as f:
        json.dump(recs, f)
    return dict(root=root, img_dir=img_dir, data_file=data_file, vid_file=vid_file, vocab=vocab, clips=allj,
                easy=jsons[0], n_clips=len(recs), vids=VIDS)


def test_u8_ingest_matches_f32_transform(corpus):
    """The same clips through the f32 host transform (ToTensor + Normalize) and through the u8 GPU ingest give the
    same fp32 logits (both paths compute (x / 255 - mean) / std in fp32)."""
    from data.infer_youtube_video_dataset import InferYoutubeClipDataset
    from train_video_segment_point import make_tokenizer, vision_transform
    from vcg_hip.build import build_two_stream
    from vcg_hip.ingest import stage_clips_u8
    tok = make_tokenizer(corpus["vocab"])
    a = InferYoutubeClipDataset(corpus["img_dir"], corpus["clips"], tok, 16, 32, transform=vision_transform(False))
    b = InferYoutubeClipDataset(corpus["img_dir"], corpus["clips"], tok, 16, 32, u8=True)
    model = build_two_stream(clip_frame_num=16, seed=123, device="cuda", precision="fp32").eval()
    xa = torch.stack([a[i][0] for i in range(2)]).cuda()
    xb = torch.stack([b[i][0] for i in range(2)])
    ids = torch.stack([a[i][1] for i in range(2)]).cuda()
    mask = torch.stack([a[i][2] for i in range(2)]).cuda()
    assert torch.equal(ids.cpu(), torch.stack([b[i][1] for i in range(2)]))
    with torch.no_grad():
        la, _ = model(xa, ids, mask)
        lb, _ = model.forward_staged(stage_clips_u8(xb, "cuda", torch.float32), ids, mask)
    torch.cuda.synchronize()
    assert (la - lb).abs().max().item() < 1e-5


def test_train_driver_on_disk(corpus, tmp_path):
    import train_video_segment_point as drv
    log = tmp_path / "tb"
    r = drv.main(TINY + ["--epoch", "1", "--batch_size", "2", "--img_dir", corpus["img_dir"], "--data_file",
                         corpus["data_file"], "--vid_file", corpus["vid_file"], "--test_clips_json", corpus["clips"],
                         "--vocab_file", corpus["vocab"], "--ckpt_path", str(tmp_path / "ck" / "checkpoint.pth"),
                         "--tensorboard_log", str(log)])
    assert r == float("-inf") or 0.0 <= r <= 1.0
    tags = set()
    for f in log.iterdir():
        if f.name == "scalars.jsonl":
            tags = {json.loads(l)["tag"] for l in f.read_text().splitlines()}
    assert {"infer_test/loss", "infer_test/auc", "infer_test/m_ap"} <= tags


def test_test_driver_on_disk(corpus, tmp_path):
    import test_video_segment_point as drv
    out = tmp_path / "res.json"
    res = drv.main(TINY + ["--img_dir", corpus["img_dir"], "--test_clips_json", corpus["clips"], "--vocab_file",
                           corpus["vocab"], "--result_file", str(out), "--precision", "fp32"])
    assert 0.0 <= res["mAP"] <= 1.0 and out.exists()
    easy = drv.main(TINY + ["--img_dir", corpus["img_dir"], "--test_clips_json", corpus["clips"],
                            "--test_easy_clips_json", corpus["easy"], "--data_type", "easy", "--vocab_file",
                            corpus["vocab"]])
    assert 0.0 <= easy["mAP"] <= 1.0
    with pytest.raises(RuntimeError):
        drv.main(TINY + ["--img_dir", corpus["img_dir"], "--test_clips_json", corpus["clips"], "--data_type", "hard"])
    with pytest.raises(RuntimeError):
        drv.main(TINY + ["--img_dir", corpus["img_dir"], "--test_clips_json", corpus["clips"], "--data_type", "x"])


def test_test_driver_batch_partition_is_the_reference_default():
    """Batch-statistics BN makes the batch partition part of the result: the driver's default is the reference's
    16 (test_video_segment_point.py:41)."""
    import test_video_segment_point as drv
    a = drv.build_parser().parse_args([])
    assert a.batch_size == 16 and a.data_type == "all"


def test_ddp_checkpoint_save_and_resume(tmp_path):
    """World 1: two epochs with a regular checkpoint every epoch, then a run to epoch 3 resumes from the newest one
    (the reference's `_(\\d+)(?:_score_[\\d.]+)?\\.pth$` rule) and trains only epoch 3."""
    import train_video_segment_ddp as drv
    os.environ.pop("WORLD_SIZE", None)
    ck = str(tmp_path / "ck") + "/"
    base = ["--clip_frame_num", "4", "--resolution", "64", "--max_text_len", "32", "--batch_size", "2", "--videos",
            "16", "--ckpt_path", ck, "--val_every", "100", "--save_every", "1"]
    drv.main(base + ["--epoch", "2"])
    names = sorted(os.listdir(ck))
    assert names == ["_1.pth", "_2.pth"], names
    path, ep = drv.find_latest_checkpoint(ck)
    assert ep == 2 and path.endswith("_2.pth")
    open(os.path.join(ck, "_10_score_0.5.pth.tmp"), "w").close()  # not a checkpoint name
    sd2 = torch.load(path, weights_only=True)
    drv.main(base + ["--epoch", "3"])
    assert sorted(n for n in os.listdir(ck) if n.endswith(".pth")) == ["_1.pth", "_2.pth", "_3.pth"]
    sd3 = torch.load(os.path.join(ck, "_3.pth"), weights_only=True)
    assert sd3["epoch"] == 3
    assert set(sd3["optimizer_state_dict"]["state"]) == set(sd2["optimizer_state_dict"]["state"])
    k = "fusion_head.head.weight"
    assert not torch.equal(sd2["model_state_dict"][k], sd3["model_state_dict"][k])


def test_bench_gpus2_rehearsal():
    """`bench.py --gpus 2` without a launcher starts its two ranks itself; here they rendezvous over gloo and share
    the box's one GPU (VCG_DIST_BACKEND=gloo), the round-end 8-GPU run uses RCCL through the same code."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env["VCG_DIST_BACKEND"] = "gloo"
    out = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--steps", "1", "--warmup",
                          "1", "--batch", "2", "--frames", "4", "--res", "112", "--tokens", "32"],
                         capture_output=True, text=True, timeout=400, cwd=REPO, env=env)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["config"]["global_batch"] == 4 and d["value"] > 0
    # the self-validating multi-GPU fields: process group, cross-rank parameter agreement, the exchange
    assert d["dist"] == {"backend": "gloo", "world_size": 2}
    assert d["params_consistent"] is True and d["params_max_abs_diff"] == 0.0
    ar = d["allreduce"]
    assert ar["buckets_per_step"] >= 5 and ar["bytes_per_step"] >= 4 * 133_000_000
    assert ar["wire_dtype"] == "fp32" and ar["exposed_ms_per_step_median"] >= 0.0
