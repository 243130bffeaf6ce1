#!/usr/bin/env python
"""Benchmark: clip-windows/sec of a TwoStream train step (TSM-ResNet-50 + BERT-base + ChapterHead,
16 frames x 224^2 + 128 tokens per window, B=64 windows per GPU, bf16, fused clip+AdamW) on 1..8
MI355X, one process per GPU (torchrun), RCCL all-reduce overlapped with the backward.

Prints ONE JSON line (rank 0).
- `roofline`: the dominant kernel (igemm_fast_kernel, the bf16 conv/linear GEMM engine), timed live with
  HIP events on the launch stream during one extra instrumented step after the timed region
  (vcg_timing_*). Each launch records its algorithmic FLOPs (2*M*N*K) and bytes (operands read once, a
  gathered A as its source tensor, outputs and fused-epilogue operands once); the bound is the one that
  dominates over the step (bytes / HBM peak vs FLOPs / MFMA peak), `achieved` the matching rate, and
  `per_launch_roofline.frac` = sum of per-launch ideal times / measured. `traffic` = its HBM bytes per
  launch from the committed PMC pass (profiles/traffic_*.json), if any.
- `roofline_step`: the whole step priced against HBM with SURVEY Appendix A's fused-minimum bytes.
- `cpu_baseline`: the CPU oracle (oracle/, test infrastructure) on a bounded sample on this host.
"""
import argparse
import json
import math
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "video-chapter-generation_amd"))
sys.path.insert(0, REPO)

METRIC = "clip-windows/sec (16f×224²+128tok) train-step at 1/2/4/8 MI355X; % HBM roofline"
METRIC_FWD = "clip-windows/sec (16f×224²+128tok) fwd-only scoring (config 2) on 1 MI355X; % HBM roofline"
HBM_PEAK_GBS = 8000.0      # MI355X HBM3E spec (MI355X_MICROARCH.md)
MFMA_PEAK_TFLOPS = {"bf16": 2500.0, "fp32": 157.3}
N_PARAMS = 133355074


# ----------------------------------------------------------------------------- roofline accounting
def resnet_counts(HW):
    """(fused-minimum activation elements, FLOPs) per frame at HWxHW."""
    elems = 0.0
    flops = 0.0
    H = HW // 2
    elems += 3 * HW * HW + 64 * H * H
    flops += 2 * 64 * H * H * 3 * 49
    Hm = (H - 1) // 2 + 1
    elems += 64 * H * H + 64 * Hm * Hm  # maxpool in + out
    H, Cin = Hm, 64
    for mid, blocks, stride in ((64, 3, 1), (128, 4, 2), (256, 6, 2), (512, 3, 2)):
        for b in range(blocks):
            s = stride if b == 0 else 1
            Ho = (H - 1) // s + 1
            elems += Cin * H * H + mid * H * H
            flops += 2 * mid * H * H * Cin
            elems += mid * H * H + mid * Ho * Ho
            flops += 2 * mid * Ho * Ho * mid * 9
            elems += mid * Ho * Ho + 4 * mid * Ho * Ho
            flops += 2 * 4 * mid * Ho * Ho * mid
            if b == 0:
                elems += Cin * H * H + 4 * mid * Ho * Ho
                flops += 2 * 4 * mid * Ho * Ho * Cin
            elems += 4 * mid * Ho * Ho  # residual read
            Cin, H = 4 * mid, Ho
    elems += 2048 * H * H  # avgpool read
    return elems, flops


def bert_counts(L, H=768, I=3072, layers=12):
    elems = layers * L * (13 * H + 2 * I) + 3 * L * H
    flops = layers * (2 * L * H * 3 * H + 4 * 12 * L * L * 64 + 2 * L * H * H + 4 * L * H * I) + 2 * H * H
    return elems, flops


def window_costs(T, HW, L, B, s_bytes, train):
    re, rf = resnet_counts(HW)
    be, bf = bert_counts(L)
    act = (re * T + be) * s_bytes
    frames = T * 3 * HW * HW * 4
    weights = N_PARAMS * s_bytes / B
    if train:
        nbytes = 3 * act + frames + (3 * N_PARAMS * s_bytes + 28 * N_PARAMS) / B
        nflops = 3 * (rf * T + bf)
    else:
        nbytes = act + frames + weights
        nflops = rf * T + bf
    return nbytes, nflops


def _per_launch(r):
    ms, ideal, nbytes, flops = r
    if ms <= 0:
        return None
    return {"frac": round(ideal / ms, 4), "ideal_ms": round(ideal, 3), "measured_ms": round(ms, 3),
            "algorithmic_gb": round(nbytes / 1e9, 3), "hbm_gbs": round(nbytes / (ms / 1e3) / 1e9, 1),
            "tflops": round(flops / (ms / 1e3) / 1e12, 1)}


def _category_frac(a, b, peak_tf):
    """Two launch categories' records taken as one: algorithmic GB/s over HBM peak (the dominant kernel's `frac`
    definition) and the per-launch roofline fraction."""
    ms, ideal, nbytes, flops = (x + y for x, y in zip(a, b))
    if ms <= 0:
        return None
    gbs = nbytes / (ms / 1e3) / 1e9
    return {"frac": round(gbs / HBM_PEAK_GBS, 4), "hbm_gbs": round(gbs, 1), "per_launch_frac": round(ideal / ms, 4),
            "tflops": round(flops / (ms / 1e3) / 1e12, 1), "measured_ms": round(ms, 3)}


def gemm_census_summary(gemms):
    """Launches per kernel (the census keys without their shapes) and in all."""
    by_kernel = {}
    for key, n in gemms.items():
        k = key.split(" M=")[0]
        by_kernel[k] = by_kernel.get(k, 0) + n
    return {"launches": sum(gemms.values()), "shapes": len(gemms), "kernels": dict(sorted(by_kernel.items())),
            "identical_to_timed_step": True}


# ----------------------------------------------------------------------------- CPU baseline
def cpu_threads():
    """Threads for the CPU baseline: the cores this process may run on, capped at 16 (a one-GPU box's CPU share;
    os.cpu_count() reports the whole host there, many times more than the share)."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 8
    return max(1, min(16, n))


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(T, HW, L, threads, mode="train", B=None, reps=None, bn="running"):
    """The oracle (oracle/model.py: fp32 CPU restatement of the reference path, test infrastructure) timed on this
    host: train = one reference train step (fwd BN-train with BERT dropout 0.1 as the GPU step runs it + CE + bwd +
    clip_grad_norm_ + AdamW), fwd = the eval forward. Median of `reps` (3) timed runs after 1 warm-up. B is a bounded
    sample (4 windows per run; 30-60 s of CPU work in all) so the default bench finishes in minutes. The per-window CPU rate barely depends on B (the CPU path has no batch-level parallelism
    beyond the threads; the round-3 sweep, profiles/r03_cpu_sweep_*.jsonl: the forward at B 64 is ~20 % SLOWER per
    window than at B 4), so a small B does not understate the CPU."""
    import torch
    from oracle import model as om
    from vcg_hip.build import build_two_stream
    from vcg_hip import synth
    B = B or 4
    reps = reps or 3
    torch.set_num_threads(threads)
    m = build_two_stream(clip_frame_num=T, dropout=0.1)
    sd = m.state_dict()
    names = [n for n, _ in m.named_parameters()]
    frames, ids, mask, labels = synth.clip_batch(B, T, HW, HW, L, seed=7)
    times = []
    for r in range(reps + 1):
        params = {n: sd[n].detach().clone().requires_grad_(mode == "train") for n in names}
        buffers = {n: sd[n].detach().clone() for n in sd if n not in params}
        t0 = time.perf_counter()
        if mode == "train":
            om.train_step(params, buffers, frames, ids, mask, labels, lr=1e-5, p_drop=0.1)
        else:
            p = dict(buffers)
            p.update(params)
            with torch.no_grad():
                om.two_stream(p, frames, ids, mask, bn_mode=bn)
        dt = time.perf_counter() - t0
        if r > 0:
            times.append(dt)
    med = sorted(times)[len(times) // 2]
    what = ("fp32 train step (fwd + bwd + clip + AdamW, BN train, dropout 0.1)" if mode == "train"
            else f"fp32 eval forward ({bn}-stat BN)")
    return {"value": round(B / med, 4), "unit": "clip-windows/sec", "cores": threads, "kind": "port",
            "cpu_model": cpu_model(), "host_cpus_visible": os.cpu_count(),
            "sample": f"oracle/ CPU {what} on B={B} windows of {T}x{HW}^2 + {L} tokens; median of {reps} timed runs "
                      f"({', '.join(f'{t:.2f}' for t in times)} s) after 1 warm-up; torch.set_num_threads({threads})",
            "why_this_sample": "B=4, not the GPU's 64: a bounded 30-60 s sample, and the CPU's per-window rate does not "
                               "grow with B (round-3 sweep, profiles/r03_cpu_sweep_*.jsonl: the forward at B=64 is ~20 % "
                               "slower per window than at B=4); 16 threads: the one-GPU box's CPU share (os.cpu_count() "
                               "reports the whole host), within 10 % of the best thread count in every sweep (4-32 "
                               "threads; 64+ ran slower)"}


# ----------------------------------------------------------------------------- config 5
def long_video_bench(args):
    """Config 5: one 1 h synthetic video (u8 frames resident in HBM), stride-1 s windows, frame gather +
    normalisation on the GPU, TwoStream scoring (eval), cut points and boundary metrics. value = windows/s of
    the GPU part (gather + forward + labels); host tokenisation is done before the timed region."""
    import numpy as np
    import torch
    import long_video as lv
    from data.synthetic_dataset import HashTokenizer
    from vcg_hip import _lib
    from vcg_hip.build import build_two_stream
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    _lib.call("vcg_init", 0)
    T, HW, L, B, F = args.frames, args.res, args.tokens, args.batch, args.video_frames
    model = build_two_stream(clip_frame_num=T, seed=123, device=dev, precision=args.precision).eval()
    if args.bn == "batch":
        from test_video_segment_point import drop_bn_running_stats
        drop_bn_running_stats(model)
    frames, timestamps, subtitles = lv.synthetic_long_video(F, HW, HW, seed=123, device=dev)
    win, idx, ids, mask = lv.window_inputs(F, T, args.stride, subtitles, HashTokenizer(), L)
    idx, ids, mask = (torch.from_numpy(a).to(dev) for a in (idx, ids, mask))
    K = args.scoring_streams
    G = args.bn_groups
    if args.bn_group_streams > 0:
        model.bn_group_streams = args.bn_group_streams
    # re-bias the random-init 2-way head (untimed, as tests/test_gpu_long_video.py does) so its decisions split
    # about evenly: otherwise every window sits on one side of 0.5, no cut point is predicted and F is 0 / undefined
    samp = torch.from_numpy(np.linspace(0, len(win) - 1, 256).astype(np.int64)).to(dev)
    with torch.no_grad():
        sc, _ = lv.score_windows(model, frames, idx[samp], ids[samp], mask[samp], B)
        pr = sc.double().clamp(1e-12, 1 - 1e-12)
        shift = -torch.log(pr / (1 - pr)).median().item()
        model.fusion_head.head.bias.data[1] += shift
        model.native_flat().refresh_shadow(force=True)
    W0 = B * max(2, K, G)
    lv.score_windows(model, frames, idx[:W0], ids[:W0], mask[:W0], B, streams=K, groups=G)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    scores, labels = lv.score_windows(model, frames, idx, ids, mask, B, streams=K, groups=G)
    torch.cuda.synchronize()
    sec = time.perf_counter() - t0
    lab = labels.cpu().tolist()
    m = lv.boundary_metrics(lab, timestamps, F, T, args.stride)
    n = len(win)
    nbytes, nflops = window_costs(T, HW, L, B, 2 if args.precision == "bf16" else 4, False)
    cpu = None
    if not args.no_cpu_baseline:
        # the oracle on the first scoring batch of the same video: a bounded sample, windows/s of the CPU forward
        from data.synthetic_dataset import normalize_frames
        from oracle import model as om
        threads = args.cpu_threads or cpu_threads()
        torch.set_num_threads(threads)
        p = {k: v.detach().float().cpu() for k, v in model.state_dict().items()}
        S = min(B, 16)  # (batch-stat BN: B = 16 is exactly the first scoring batch)
        img = normalize_frames(frames[idx[:S].reshape(-1)].cpu().numpy().reshape(-1, T, HW, HW, 3))
        ts = []
        for r in range(3):
            t1 = time.perf_counter()
            with torch.no_grad():
                om.two_stream(p, img, ids[:S].cpu(), mask[:S].cpu(), bn_mode=args.bn)
            if r:
                ts.append(time.perf_counter() - t1)
        runs = ", ".join(f"{t:.2f}" for t in ts)
        cpu = {"value": round(S / sorted(ts)[len(ts) // 2], 4), "unit": "clip-windows/sec", "cores": threads,
               "kind": "port", "cpu_model": cpu_model(), "host_cpus_visible": os.cpu_count(),
               "sample": f"oracle/ CPU fp32 forward ({args.bn}-stat BN) of the first {S} windows of "
                         f"the same video; median of 2 timed runs ({runs} s) after 1 warm-up; frame gather and "
                         f"normalisation excluded; torch.set_num_threads({threads})"}
    print(json.dumps({
        "metric": f"clip-windows/sec long-video inference (config 5: 1 h video, stride-{args.stride} s windows)",
        "value": round(n / sec, 3), "unit": "clip-windows/sec", "n_gpus": 1, "windows": n, "seconds": round(sec, 3),
        "higher_is_better": True, "dtype": args.precision,
        "data": "synthetic 1 fps video (seeded u8 frames in HBM, random-init weights)",
        "config": {"workload": f"{F} frames {HW}^2, T={T}, L={L}, stride {args.stride} s, batch {B}, "
                               f"{args.bn}-stats BN" + (f", batches on {K} streams" if K > 1 else "")
                               + (f", {G} batches per forward (per-batch statistics)" if G > 1 else ""),
                   "bn": args.bn, "stride": args.stride, "scoring_streams": K, "bn_groups": G,
                   "frames": F, "clip_frame_num": T, "seq_len": L, "resolution": HW},
        "cpu_baseline": cpu,
        "roofline_step": {"bound": "hbm", "achieved": round(nbytes * n / sec / 1e9, 2), "peak": HBM_PEAK_GBS,
                          "unit": "GB/s", "frac": round(nbytes * n / sec / 1e9 / HBM_PEAK_GBS, 4),
                          "mfma_tflops": round(nflops * n / sec / 1e12, 2)},
        "boundary": {k: m[k] for k in ("recall", "recall_3", "recall_5", "precision", "precision_3", "precision_5",
                                       "f", "f_3", "f_5")},
        "head_calibration": {"logit1_bias_shift": round(shift, 5), "sample_windows": 256,
                             "positive_share": round(sum(lab) / max(len(lab), 1), 4),
                             "note": "random-init head re-biased (untimed) so about half the windows score positive"}}),
        flush=True)


# ----------------------------------------------------------------------------- multi-GPU evidence
def ddp_evidence(reducer, flat, exposed_ms, transport):
    """Collective over all ranks (every rank calls it after the timed steps): what rank 0's line carries for a
    world > 1 run so that the run validates itself -- the process group as seen from inside (backend, world size),
    cross-rank parameter agreement (max |param - rank-0 param| over the whole flat buffer, all-reduced with MAX:
    0 when the ranks stayed in lockstep, as DDP guarantees), and the gradient exchange (buckets and bytes one
    backward put on the wire, wire dtype, and the exposed communication time: from the end of the backward's
    work on the step's stream to the reducer's finish() having joined every collective, timed on that stream).
    Replaces the reference's DDP wiring, train_video_segment_ddp.py:148,261-263,339."""
    import torch.distributed as dist
    from vcg_hip.ddp import params_max_divergence
    div = params_max_divergence(flat)
    ex = sorted(exposed_ms) or [float("nan")]
    return {"dist": {"backend": str(dist.get_backend()), "world_size": dist.get_world_size()},
            "params_consistent": div == 0.0, "params_max_abs_diff": div,
            "allreduce": {"transport": transport, "op": "sum (1/world folded into AdamW)",
                          "bucket_bytes": reducer.bucket_elems * 4,
                          "buckets_per_step": reducer.last_step["buckets"],
                          "bytes_per_step": reducer.last_step["bytes"],
                          "wire_dtype": "bf16" if reducer.wire is not None else "fp32",
                          "exposed_ms_per_step_median": round(ex[len(ex) // 2], 4),
                          "exposed_ms_per_step_max": round(ex[-1], 4),
                          "exposed_timing": "stream events: backward done -> finish() joined (timed steps)"}}


def cpu_ddp_rehearsal(steps=3):
    """--launch-check's model-free DDP step on the CPU (gloo): a small Linear stack in a FlatParams buffer, each
    rank on its own inputs, gradients reported to GradAllReducer in backward order with small buckets, a plain SGD
    update with the 1/world average -- the same reducer and ddp_evidence() the GPU bench line uses."""
    import torch
    import torch.distributed as dist
    from vcg_hip.ddp import GradAllReducer, broadcast_parameters
    from vcg_hip.flat import FlatParams
    torch.manual_seed(dist.get_rank())  # ranks start apart: broadcast_parameters must align them
    net = torch.nn.Sequential(torch.nn.Linear(64, 256), torch.nn.ReLU(), torch.nn.Linear(256, 256), torch.nn.ReLU(),
                              torch.nn.Linear(256, 8))
    flat = FlatParams(list(net.named_parameters()), "cpu")

    class _M(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.net = net

        def native_flat(self):
            return flat
    broadcast_parameters(_M())
    red = GradAllReducer(flat, bucket_bytes=64 << 10)
    world = dist.get_world_size()
    gen = torch.Generator().manual_seed(1000 + dist.get_rank())
    exposed = []
    layers = [m for m in net if isinstance(m, torch.nn.Linear)]
    for _ in range(steps):
        flat.zero_grad()
        x = torch.randn(32, 64, generator=gen)
        net(x).square().mean().backward()
        for lin in reversed(layers):  # the engines' backward-order reports
            red([lin.weight, lin.bias])
        t0 = time.perf_counter()
        red.finish()
        exposed.append(1e3 * (time.perf_counter() - t0))
        with torch.no_grad():
            flat.data.add_(flat.grad, alpha=-0.1 / world)
    return ddp_evidence(red, flat, exposed, "torch.distributed")


# ----------------------------------------------------------------------------- launcher
def _free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n):
    """Run this same command as an n-rank torch.distributed.run job (rendezvous on 127.0.0.1) in a child process
    and return its exit status. Rank 0 of the job prints the JSON line."""
    import subprocess
    port = os.environ.get("MASTER_PORT") or str(_free_port())
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("OMP_NUM_THREADS", "4")
    return subprocess.call(cmd, env=env)


def launch_check(args, world, rank):
    """The launch path without the model: the ranks rendezvous (gloo), count themselves with an all-reduce and
    rank 0 prints n_gpus and the local ranks it saw (tests/test_cpu_bench_launch.py)."""
    import torch
    import torch.distributed as dist
    if world > 1:
        dist.init_process_group("gloo")
    t = torch.tensor([1, int(os.environ.get("LOCAL_RANK", "0"))], dtype=torch.int64)
    seen = [torch.zeros_like(t) for _ in range(world)]
    if world > 1:
        dist.all_gather(seen, t)
    else:
        seen = [t]
    ev = cpu_ddp_rehearsal() if world > 1 else {}
    if rank == 0:
        print(json.dumps({"metric": METRIC, "n_gpus": int(sum(int(s[0]) for s in seen)),
                          "local_ranks": [int(s[1]) for s in seen], "launch_check": True, **ev}), flush=True)
    if world > 1:
        dist.destroy_process_group()


# ----------------------------------------------------------------------------- main
def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=None,
                    help="clip windows per GPU (default 64; 16 with --bn batch, the test driver's batch)")
    ap.add_argument("--frames", type=int, default=16)
    ap.add_argument("--res", type=int, default=224)
    ap.add_argument("--tokens", type=int, default=128)
    ap.add_argument("--precision", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--mode", default="train", choices=["train", "fwd", "long_video"],
                    help="long_video: BASELINE config 5 (1 h synthetic video, stride-1 s windows, on-GPU frame "
                         "ingest, end-to-end boundary metrics), 1 GPU")
    ap.add_argument("--video-frames", type=int, default=3600)
    ap.add_argument("--stride", type=int, default=1, help="long_video: window stride in s (the reference's own: 4)")
    ap.add_argument("--scoring-streams", type=int, default=1,
                    help="long_video: scoring batches round-robin over this many HIP streams (long_video.score_windows); "
                         "fwd: a step scores this many batches of --batch windows, one per HIP stream")
    ap.add_argument("--bn-groups", type=int, default=1,
                    help="batch-statistics scoring (--bn batch): this many batches of --batch windows form ONE forward "
                         "with per-batch BatchNorm statistics (TwoStream.bn_group: the trunk per batch, BERT and the "
                         "head once over all of them); fwd: a step is that forward; long_video: score_windows(groups)")
    ap.add_argument("--bn", default="running", choices=["running", "batch"],
                    help="scoring modes (fwd / long_video): BN with running statistics (model.eval(), the trainer's "
                         "val and convert2vision_emb) or with the batch's statistics (test_video_segment_point.py:"
                         "116-122, which scores batches of 16 windows: pass --batch 16)")
    ap.add_argument("--bn-group-streams", type=int, default=0,
                    help="with --bn-groups: the groups' trunks round-robin on this many HIP streams "
                         "(TwoStream.bn_group_streams; 0: the model's default)")
    ap.add_argument("--full-text", action="store_true",
                    help="synthetic subtitles fill all --tokens positions (default: n_valid uniform in [L/2, L], "
                         "vcg_hip.synth.clip_batch): the BERT work without any padded rows to drop")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=0)
    ap.add_argument("--no-roofline-step", action="store_true",
                    help="skip the instrumented step after the timed region (profiling runs: the trace then ends with "
                         "the timed steps); the line then has no dominant-kernel roofline")
    ap.add_argument("--one-stream", action="store_true",
                    help="every kernel on one HIP stream (BERT, the trunk's weight gradients and downsample branch "
                         "inline): the one-stream rocprof profiles, whose per-kernel durations are unshared")
    ap.add_argument("--launch-check", action="store_true",
                    help="rehearse the rank launch only (gloo, no GPU): every rank joins the process group and "
                         "rank 0 prints the line's n_gpus / rank layout")
    args = ap.parse_args()
    if args.batch is None:
        args.batch = 16 if (args.bn == "batch" and args.mode != "train") else 64

    if args.bn_groups > 1 and (args.bn != "batch" or args.mode == "train" or args.scoring_streams > 1):
        raise SystemExit("bench.py: --bn-groups applies to batch-statistics scoring (--bn batch, fwd / long_video) "
                         "on one stream")
    if args.mode == "long_video" and args.gpus > 1:
        raise SystemExit("bench.py: --mode long_video is a one-GPU benchmark (config 5); run it with --gpus 1")
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # `bench.py --gpus N` without a launcher: start the N rank processes ourselves, one per GPU, as the
        # reference's DDP driver does with mp.spawn (train_video_segment_ddp.py:599-608). This process has not
        # touched the GPU (torch is not even imported yet), and the ranks are fresh child processes, not an exec.
        return launch_ranks(args.gpus)
    import torch
    import torch.distributed as dist

    if args.mode == "long_video":
        return long_video_bench(args)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}: the launcher and the flag disagree")
    if args.launch_check:
        return launch_check(args, world, rank)
    # one process per GPU; VCG_DIST_BACKEND=gloo + more ranks than GPUs only for rehearsing the DDP path on a
    # one-GPU box (ranks then share devices round-robin); the benchmark itself is RCCL ("nccl") over xGMI
    backend = os.environ.get("VCG_DIST_BACKEND", "nccl")
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if backend != "nccl":
        local %= max(1, torch.cuda.device_count())
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    from vcg_hip import _lib, ops, synth
    from vcg_hip.build import build_two_stream
    from vcg_hip.ddp import BufferBroadcaster, GradAllReducer, broadcast_parameters
    from vcg_hip.functions import cross_entropy

    _lib.call("vcg_init", local)
    B, T, HW, L = args.batch, args.frames, args.res, args.tokens
    torch.manual_seed(123)
    model = build_two_stream(clip_frame_num=T, seed=123, device=dev, precision=args.precision)
    model.train(args.mode == "train")
    if args.one_stream:
        from vcg_hip.trunk import ResNetTrunk
        model.overlap_streams = ResNetTrunk.wgrad_stream = ResNetTrunk.ds_stream = False
    if args.mode == "fwd" and args.bn == "batch":
        from test_video_segment_point import drop_bn_running_stats
        drop_bn_running_stats(model)

    class Cfg:
        weight_decay = 0.01
        learning_rate = 1e-5
        betas = (0.9, 0.95)
    opt = model.configure_optimizers(Cfg)
    flat = model.native_flat()
    # DDP transport: torch.distributed RCCL (default) or libvcg_hip's RCCL C ABI on a side stream (VCG_COMM=native);
    # fp32 wire as the reference's DDP, or bf16 (VCG_DDP_WIRE=bf16)
    comm = None
    if world > 1 and os.environ.get("VCG_COMM", "") == "native":
        from vcg_hip.comm import NativeComm
        comm = NativeComm()
    wire = torch.bfloat16 if os.environ.get("VCG_DDP_WIRE", "") == "bf16" else None
    reducer = GradAllReducer(flat, comm=comm, wire_dtype=wire)
    bufsync = None
    if world > 1:
        broadcast_parameters(model)
        model.set_grad_hooks(reducer)
        opt.grad_scale = 1.0 / world
        bufsync = BufferBroadcaster(model, comm=comm)  # DDP broadcast_buffers: rank 0's BN stats each forward
    # fwd with --scoring-streams K > 1: a step scores K batches of B windows, batch k on HIP stream k (batch 0 on the
    # main stream first in the first step, so one-time weight preparation is ordered before the others): the
    # batch-statistics mode scores batches of 16 (BN couples only the windows of one batch), which underfill the chip
    K = args.scoring_streams if args.mode == "fwd" else 1
    # fwd with --bn-groups G: a step is ONE forward over G batches of B windows, BatchNorm statistics per batch
    G = args.bn_groups if args.mode == "fwd" else 1
    if G > 1:
        model.bn_group = B
        if args.bn_group_streams > 0:
            model.bn_group_streams = args.bn_group_streams
    frames, ids, mask, labels = synth.clip_batch(B * K * G, T, HW, HW, L, seed=123 + rank, device=dev)
    if args.full_text:  # every window's subtitle fills all L tokens (no padding for BERT to drop)
        ids[ids == 0] = 1000
        mask.fill_(1)
    chunks = [(frames[k * B:(k + 1) * B], ids[k * B:(k + 1) * B], mask[k * B:(k + 1) * B]) for k in range(K)]
    pool = [torch.cuda.current_stream(dev)] + [torch.cuda.Stream(device=dev) for _ in range(K - 1)]
    comm_events = None  # [(backward done, finish joined)] per timed step (world > 1)
    prepared = []

    def step():
        if args.mode == "fwd":
            with torch.no_grad():
                if K == 1:
                    model(frames, ids, mask)
                    return
                main = pool[0]
                if not prepared:  # the first forward prepares the weights on the main stream
                    model(*chunks[0])
                for s_ in pool[1:]:
                    s_.wait_stream(main)
                for k, (f_, i_, m_) in enumerate(chunks):
                    if k == 0 and not prepared:
                        continue
                    with torch.cuda.stream(pool[k]):
                        model(f_, i_, m_)
                prepared.append(True)
                for s_ in pool[1:]:
                    main.wait_stream(s_)
            return
        opt.zero_grad()
        if bufsync is not None:
            bufsync()
        logits, prob = model(frames, ids, mask)
        loss = cross_entropy(logits, labels)
        loss.backward()
        if comm_events is not None:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            reducer.finish()
            e1.record()
            comm_events.append((e0, e1))
        else:
            reducer.finish()
        opt.clip_and_step(1.0)

    from vcg_hip.trunk import ResNetTrunk
    # the per-block path census (which bn3 fold / y3-drop / GEMM-pass variant every bottleneck ran) of the last
    # warm-up step: the timed steps run the same path; the instrumented step below must too
    # and the GEMM census (which kernel ran which GEMM shape, every GEMM-class launch of the step: libvcg_hip's
    # vcg_gemm_census) of the same step: the instrumented step below must match it launch for launch
    timed_census = timed_gemms = None
    for i in range(args.warmup):
        last = i == args.warmup - 1
        if last and args.mode == "train":
            ResNetTrunk.census = []
        if last:
            ops.gemm_census_enable(True)
        step()
        if last:
            timed_gemms = ops.gemm_census()
            ops.gemm_census_enable(False)
        timed_census, ResNetTrunk.census = ResNetTrunk.census, None
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record()
    enq = []  # host time to enqueue each step (launches are asynchronous: << ms_per_step unless the host stalls)
    import gc
    gc0 = [g["collections"] for g in gc.get_stats()]
    ms0 = torch.cuda.memory_stats()
    if world > 1 and args.mode == "train":
        comm_events = []
    for _ in range(args.steps):
        te = time.perf_counter()
        step()
        enq.append(time.perf_counter() - te)
    ev1.record()
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    ms1 = torch.cuda.memory_stats()
    exposed = [a.elapsed_time(b) for a, b in comm_events] if comm_events else []
    comm_events = None
    host_diag = {"slowest_step": int(max(range(len(enq)), key=lambda i: enq[i])),
                 "gc_collections": [g["collections"] - c for g, c in zip(gc.get_stats(), gc0)],
                 "device_allocs": ms1.get("num_device_alloc", 0) - ms0.get("num_device_alloc", 0),
                 "device_frees": ms1.get("num_device_free", 0) - ms0.get("num_device_free", 0),
                 "alloc_retries": ms1.get("num_alloc_retries", 0) - ms0.get("num_alloc_retries", 0),
                 "reserved_gb": round(torch.cuda.memory_reserved() / 2**30, 1)}
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    ms = ev0.elapsed_time(ev1) / args.steps
    ms = max(ms, wall * 1000.0 / args.steps)
    # one extra (untimed) step with every fast-GEMM launch bracketed by HIP events; BERT runs on the trunk's
    # stream for this step, so a launch's duration is the kernel's own (not shared with a concurrent kernel)
    sides = (model.overlap_streams, ResNetTrunk.wgrad_stream, ResNetTrunk.ds_stream)
    # (and the weight gradients / downsample convs / weight re-layout on the trunk's stream)
    model.overlap_streams = ResNetTrunk.wgrad_stream = ResNetTrunk.ds_stream = False
    ops.timing_enable(True)
    census = gemm_census = None
    if not args.no_roofline_step:
        ResNetTrunk.census = [] if timed_census is not None else None
        ops.gemm_census_enable(timed_gemms is not None)
        step()
        inst_census, ResNetTrunk.census = ResNetTrunk.census, None
        if timed_gemms is not None:
            inst_gemms = ops.gemm_census()
            ops.gemm_census_enable(False)
            # every GEMM of the instrumented step on the kernel the timed steps used (no silent fallback between them)
            assert inst_gemms == timed_gemms, ("instrumented step ran other GEMM kernels than the timed steps",
                                               sorted(set(inst_gemms.items()) ^ set(timed_gemms.items()))[:8])
            gemm_census = gemm_census_summary(timed_gemms)
        if timed_census is not None:
            # the one-stream instrumented step must run the timed step's kernels (bn3 folds, y3 drops, GEMM passes)
            assert inst_census == timed_census, ("instrumented step ran another per-block path than the timed steps",
                                                 timed_census, inst_census)
            census = {"blocks_fwd": sum(e[0] == "fwd" for e in timed_census),
                      "blocks_bwd": sum(e[0] == "bwd" for e in timed_census),
                      "bn3_fold_bwd": sum(e[0] == "bwd" and e[3]["fold_dgrad"] for e in timed_census),
                      "y3_drop": sum(e[0] == "fwd" and e[3]["y3_drop"] for e in timed_census),
                      "identical_to_timed_step": True}
    torch.cuda.synchronize()
    # the dominant kernel: the bf16 fast engine, or the generic engine (exact fp32 MFMA) in the parity precision
    dom_id, dom_name = ((ops.TIMING_FAST_GEMM, "igemm_fast_kernel") if args.precision == "bf16"
                        else (ops.TIMING_GENERIC_GEMM, "igemm_kernel"))
    k_ms, k_n, k_fl = ops.timing_query(dom_id)
    peak_tf = MFMA_PEAK_TFLOPS[args.precision]
    rl = {kid: ops.timing_roofline(kid, peak_tf, HBM_PEAK_GBS) for kid in (dom_id, ops.TIMING_WGRAD,
                                                                           ops.TIMING_WIDE_GEMM)}
    wide_n = ops.timing_query(ops.TIMING_WIDE_GEMM)[1]
    ops.timing_enable(False)
    model.overlap_streams, ResNetTrunk.wgrad_stream, ResNetTrunk.ds_stream = sides
    kern = {"ms": k_ms, "launches": k_n, "flops": k_fl}
    ddp = {}
    if world > 1:
        t = torch.tensor([ms], device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        ms = float(t.item())
        if args.mode == "train":
            ddp = ddp_evidence(reducer, flat, exposed, "libvcg_hip RCCL C ABI" if comm is not None else
                               "torch.distributed")

    if rank == 0:
        windows = B * K * G * world
        value = windows / (ms / 1000.0)
        s_bytes = 2 if args.precision == "bf16" else 4
        nbytes, nflops = window_costs(T, HW, L, B, s_bytes, args.mode == "train")
        achieved = nbytes * B * K * G / (ms / 1000.0) / 1e9  # per GPU
        tflops = nflops * B * K * G / (ms / 1000.0) / 1e12
        traffic = kern_traffic = mfma_busy = None
        tf = os.path.join(REPO, "profiles", f"traffic_{args.mode}_{args.precision}_b{B}.json")
        if os.path.exists(tf):
            with open(tf) as f:
                tj = json.load(f)
            traffic = tj.get("hbm_bytes_per_step")
            kern_traffic = tj.get(dom_name, {}).get("hbm_bytes_per_launch")
        mf = os.path.join(REPO, "profiles", f"mfma_{args.mode}_{args.precision}_b{B}.json")
        if os.path.exists(mf):  # PMC SQ_VALU_MFMA_BUSY_CYCLES pass (tools/mfma.sh)
            with open(mf) as f:
                mfma_busy = json.load(f).get(dom_name)
        dom = None
        if kern["launches"]:
            # the dominant kernel's bound from its aggregate arithmetic intensity over the step: algorithmic
            # bytes / HBM peak vs algorithmic FLOPs / MFMA peak (ridge ~312 flop/B in bf16)
            r_ms, r_ideal, r_bytes, r_flops = rl[dom_id]
            k_tf = kern["flops"] / (kern["ms"] / 1e3) / 1e12
            k_gbs = r_bytes / (kern["ms"] / 1e3) / 1e9
            hbm_bound = r_bytes / (HBM_PEAK_GBS * 1e9) >= r_flops / (peak_tf * 1e12)
            dom = {"kernel": dom_name, "bound": "hbm" if hbm_bound else "mfma",
                   "achieved": round(k_gbs if hbm_bound else k_tf, 2),
                   "peak": HBM_PEAK_GBS if hbm_bound else peak_tf, "unit": "GB/s" if hbm_bound else "TFLOP/s",
                   "frac": round((k_gbs / HBM_PEAK_GBS) if hbm_bound else (k_tf / peak_tf), 4),
                   "traffic": kern_traffic,
                   "algorithmic_bytes_per_launch": round(r_bytes / kern["launches"]),
                   "arithmetic_intensity_flop_per_byte": round(r_flops / max(r_bytes, 1.0), 1),
                   "mfma_view": {"achieved": round(k_tf, 2), "peak": peak_tf, "unit": "TFLOP/s",
                                 "frac": round(k_tf / peak_tf, 4)},
                   "mfma_busy_pmc": mfma_busy,
                   "launches_per_step": kern["launches"], "avg_launch_us": round(kern["ms"] * 1e3 / kern["launches"], 2),
                   "gflop_per_launch": round(kern["flops"] / kern["launches"] / 1e9, 3),
                   "share_of_step": round(kern["ms"] / ms, 4),
                   # the same launches against their own roofline: ideal = sum of max(flops / MFMA peak,
                   # algorithmic bytes / HBM peak) per launch
                   "per_launch_roofline": _per_launch(rl[dom_id]),
                   "wgrad_fast_kernel": _per_launch(rl[ops.TIMING_WGRAD]),
                   # the dense bf16 GEMMs of BERT's Linear layers and the downsample input gradient
                   "gemm_wide_kernel": ({**_per_launch(rl[ops.TIMING_WIDE_GEMM]), "launches_per_step": wide_n}
                                        if _per_launch(rl[ops.TIMING_WIDE_GEMM]) else None),  # (fp32: none)
                   # round 4's category: every launch of the 128 x 128 / 256-tile engines AND the wide engine's (BERT's
                   # dense GEMMs were on the 128 x 128 engine then), so that moving GEMMs between engines does not
                   # read as kernel speed
                   "frac_round4_category": _category_frac(rl[dom_id], rl[ops.TIMING_WIDE_GEMM], peak_tf),
                   "path_census": census,
                   "gemm_census": gemm_census,
                   "timing": "HIP events around each launch on its stream, one instrumented step (no BERT side "
                             "stream in that step: unshared launch durations); the category also holds the 256-tile "
                             "engine's launches (rocprof name gemm256_kernel: the layer-4 3x3 forward convs)"}
        out = {
            "metric": METRIC if args.mode == "train" else METRIC_FWD, "value": round(value, 3), "unit": "clip-windows/sec", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": args.precision,
            "data": "synthetic (seeded clip windows generated in HBM; random-init weights)",
            "config": {"workload": f"TwoStream {args.mode} step: TSM-ResNet-50 + BERT-base + ChapterHead(mlp), "
                                   f"B={B} windows/GPU of {T}x{HW}^2 frames + {L} tokens"
                                   + (", fused clip+AdamW" if args.mode == "train" else ""),
                       "global_batch": windows, "seq_len": L, "frames": T, "resolution": HW,
                       "text_fill": "full" if args.full_text else "n_valid ~ U[L/2, L]",
                       **({"batches_per_step": K, "batch": B, "scoring_streams": K} if K > 1 else {}),
                       **({"batches_per_step": G, "batch": B, "bn_groups": G} if G > 1 else {}),
                       "parallelism": f"dp{world}", **({"bn": args.bn} if args.mode == "fwd" else {})},
            "roofline": dom,
            **ddp,
            "host": {"enqueue_ms_per_step_median": round(1e3 * sorted(enq)[len(enq) // 2], 3),
                     "enqueue_ms_per_step_max": round(1e3 * max(enq), 3), **host_diag},
            "roofline_step": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                         "scope": "whole step (all kernels) vs SURVEY App. A fused-minimum bytes "
                                  f"({nbytes / 1e9:.3f} GB/window)",
                         "mfma_tflops": round(tflops, 2), "mfma_frac": round(tflops / MFMA_PEAK_TFLOPS[args.precision], 4)},
        }
        if world == 1 and not args.no_cpu_baseline:
            threads = args.cpu_threads or cpu_threads()
            try:
                out["cpu_baseline"] = cpu_baseline(T, HW, L, threads, args.mode, bn=args.bn)
            except Exception as e:  # the GPU number stands on its own; report why the baseline is missing
                out["cpu_baseline"] = {"value": None, "error": repr(e)}
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    sys.exit(main() or 0)
