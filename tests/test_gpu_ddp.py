"""The data-parallel train step on the GPU with two ranks (gloo on one device: the pool's boxes have one GPU;
the round-end 8-GPU run uses RCCL over xGMI through the same code). Exercises the overlapped bucket
all-reduce with the BERT side stream: both ranks see identical inputs, so after a step their parameters must
be bit-identical to each other and equal (to fp32 rounding of (g + g) / 2 = g) to a single-process step."""
import os
import socket

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _step(model, frames, ids, mask, labels, reducer, opt):
    from vcg_hip.functions import cross_entropy
    opt.zero_grad()
    loss = cross_entropy(model(frames, ids, mask)[0], labels)
    loss.backward()
    if reducer is not None:
        reducer.finish()
    opt.clip_and_step(1.0)
    return loss


def _build(stats):
    from vcg_hip.build import build_two_stream
    from vcg_hip import synth
    m = build_two_stream(clip_frame_num=4, seed=123, device="cuda", precision="bf16", bn_stats=stats,
                         dropout=0.0).train()

    class Cfg:
        weight_decay = 0.01
        learning_rate = 1e-4
        betas = (0.9, 0.95)
    return m, m.configure_optimizers(Cfg), synth.clip_batch(2, 4, 112, 112, 32, seed=9, device="cuda")


def _worker(rank, world, port, out):
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                    "video-chapter-generation_amd"))
    import torch.distributed as dist
    from vcg_hip.ddp import GradAllReducer, broadcast_parameters
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    stats = dict(np.load(os.path.join(GOLD, "bn_running_stats.npz"), allow_pickle=False))
    m, opt, (frames, ids, mask, labels) = _build(stats)
    broadcast_parameters(m)
    red = GradAllReducer(m.native_flat(), bucket_bytes=int(os.environ.get("VCG_TEST_BUCKET", 8 << 20)), record=True)
    m.set_grad_hooks(red)
    opt.grad_scale = 1.0 / world
    from vcg_hip.functions import cross_entropy
    opt.zero_grad()
    cross_entropy(m(frames, ids, mask)[0], labels).backward()
    red.finish()
    torch.cuda.synchronize()
    # overlap evidence from the real engines: buckets went out while the backward was still reporting final
    # parameters (the first flush precedes the last hook; at most the final flush comes after it)
    kinds = [e[0] for e in red.log]
    last_hook = max(i for i, k in enumerate(kinds) if k == "hook")
    out[f"overlap{rank}"] = (kinds.count("flush") >= 3 and kinds.index("flush") < last_hook
                             and sum(1 for i, k in enumerate(kinds) if k == "flush" and i > last_hook) <= 1)
    out[f"grad{rank}"] = m.native_flat().grad.cpu().clone()
    opt.clip_and_step(1.0)
    _step(m, frames, ids, mask, labels, red, opt)
    torch.cuda.synchronize()
    out[rank] = m.native_flat().data.cpu()
    dist.destroy_process_group()


def test_ddp_two_ranks_match_single_process():
    import torch.multiprocessing as mp
    stats = dict(np.load(os.path.join(GOLD, "bn_running_stats.npz"), allow_pickle=False))
    m, opt, (frames, ids, mask, labels) = _build(stats)
    from vcg_hip.functions import cross_entropy
    opt.zero_grad()
    cross_entropy(m(frames, ids, mask)[0], labels).backward()
    torch.cuda.synchronize()
    g_single = m.native_flat().grad.cpu().clone()
    opt.clip_and_step(1.0)
    _step(m, frames, ids, mask, labels, None, opt)
    torch.cuda.synchronize()
    single = m.native_flat().data.cpu()
    ctx = mp.get_context("spawn")
    with ctx.Manager() as mgr:
        out = mgr.dict()
        port = _port()
        procs = [ctx.Process(target=_worker, args=(r, 2, port, out)) for r in range(2)]
        for p in procs:
            p.start()
        for p in procs:
            p.join(timeout=240)
        assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
        r0, r1 = out[0], out[1]
        g0 = out["grad0"]
        assert out["overlap0"] and out["overlap1"], "buckets were not issued during the backward"
    f = m.native_flat()
    bad = [n for n, p in m.named_parameters()
           if not torch.equal(g0[f.offset_of(p):f.offset_of(p) + p.numel()],
                              2 * g_single[f.offset_of(p):f.offset_of(p) + p.numel()])]
    assert not bad, f"{len(bad)} reduced gradients != 2 x single-process, e.g. {bad[:8]}"
    assert torch.equal(r0, r1), "ranks diverged"
    # a second single-process run: the step itself is deterministic
    m2, opt2, _ = _build(stats)
    for _ in range(2):
        _step(m2, frames, ids, mask, labels, None, opt2)
    torch.cuda.synchronize()
    assert torch.equal(m2.native_flat().data.cpu(), single), "the single-process step is not deterministic"
    diff = (r0 - single).abs()
    d = diff.max().item()
    if d > 1e-6 * (1 + single.abs().max().item()):
        f = m.native_flat()
        worst = sorted(((diff[f.offset_of(p):f.offset_of(p) + p.numel()].max().item(), n)
                        for n, p in m.named_parameters()), reverse=True)[:8]
        raise AssertionError(f"DDP != single process by {d:.3e}; worst params {worst}")


def test_native_comm_world1_and_reducer():
    """libvcg_hip's RCCL C ABI (vcg_comm_init / vcg_allreduce_bucket / vcg_broadcast_bucket, comm.hip) on this
    one-GPU box: a world-1 communicator (SUM over one rank = identity), and GradAllReducer driving it from the real
    backward on a side stream, fp32 and bf16 wire (the multi-rank run is the round-end 8-GPU bench)."""
    from vcg_hip import synth
    from vcg_hip.build import build_two_stream
    from vcg_hip.comm import NativeComm, unique_id
    from vcg_hip.ddp import BufferBroadcaster, GradAllReducer
    from vcg_hip.functions import cross_entropy
    torch.cuda.set_device(0)
    comm = NativeComm(rank=0, world=1, uid=unique_id())
    try:
        for dt in (torch.float32, torch.bfloat16):
            t = torch.randn(1 << 20, device="cuda").to(dt)
            t0 = t.clone()
            side = torch.cuda.Stream()
            side.wait_stream(torch.cuda.current_stream())
            comm.all_reduce(t, stream=side)
            comm.broadcast(t, root=0, stream=side)
            torch.cuda.current_stream().wait_stream(side)
            torch.cuda.synchronize()
            assert torch.equal(t, t0), dt
        stats = dict(np.load(os.path.join(GOLD, "bn_running_stats.npz"), allow_pickle=False))
        frames, ids, mask, labels = synth.clip_batch(2, 4, 112, 112, 32, seed=9, device="cuda")
        grads = {}
        for wire in (None, "plain", torch.bfloat16):
            m = build_two_stream(clip_frame_num=4, seed=123, device="cuda", precision="bf16", bn_stats=stats,
                                 dropout=0.0).train()
            f = m.native_flat()
            red = None
            if wire is not None:
                red = GradAllReducer(f, bucket_bytes=8 << 20, comm=comm, record=True,
                                     wire_dtype=None if wire == "plain" else wire)
                red.enabled = True  # world 1: exercise the path anyway
                m.set_grad_hooks(red)
                BufferBroadcaster(m, comm=comm)()
            f.zero_grad()
            cross_entropy(m(frames, ids, mask)[0], labels).backward()
            if red is not None:
                red.finish()
                kinds = [e[0] for e in red.log]
                last_hook = max(i for i, k in enumerate(kinds) if k == "hook")
                assert kinds.count("flush") >= 3 and kinds.index("flush") < last_hook
            torch.cuda.synchronize()
            grads[wire] = f.grad.clone()
        assert torch.equal(grads[None], grads["plain"])
        assert torch.equal(grads[torch.bfloat16], grads[None].bfloat16().float())
    finally:
        comm.close()
