"""world_size-2 gloo tests (CPU) of the data-parallel exchange in vcg_hip/ddp.py: bucketed
all-reduce of a flat gradient buffer as parameters are reported final in backward order,
no_sync-style micro-steps, rank-0 parameter broadcast and the metric gather."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


class _FakeFlat:
    """The pieces of vcg_hip.flat.FlatParams the reducer uses: a flat grad and offsets."""

    def __init__(self, sizes, seed):
        self.offsets, o = [], 0
        for n in sizes:
            self.offsets.append(o)
            o += (n + 255) // 256 * 256
        self.total = o
        g = torch.Generator().manual_seed(seed)
        self.grad = torch.randn(o, generator=g)
        self.data = torch.randn(o, generator=g)
        self.params = [torch.empty(n) for n in sizes]
        self._off = {id(p): off for p, off in zip(self.params, self.offsets)}
        self.refreshed = False

    def offset_of(self, p):
        return self._off[id(p)]

    def refresh_shadow(self, force=False):
        self.refreshed = True


class _FakeModel(torch.nn.Module):
    def __init__(self, flat):
        super().__init__()
        self._f = flat
        self.register_buffer("running_mean", torch.full((4,), float(dist.get_rank())))

    def native_flat(self):
        return self._f


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from vcg_hip.ddp import GradAllReducer, all_gather_object, broadcast_parameters
        sizes = [1000, 300, 70000, 5, 2048, 77777, 256, 1]
        flat = _FakeFlat(sizes, seed=100 + rank)
        local = flat.grad.clone()
        red = GradAllReducer(flat, bucket_bytes=64 * 1024)      # small buckets: many flushes
        # backward order: last parameters first, in groups (as the engines report them)
        groups = [[flat.params[7], flat.params[6]], [flat.params[5]], [flat.params[4], flat.params[3]],
                  [flat.params[2]], [flat.params[1], flat.params[0]]]
        for g in groups:
            red(g)
        red.finish()
        total = torch.zeros_like(local)
        for r in range(world):
            total += _FakeFlat(sizes, seed=100 + r).grad
        ok_sum = torch.allclose(flat.grad, total, rtol=0, atol=1e-5)
        # disabled reducer (accumulation micro-step) leaves the local gradient alone
        before = flat.grad.clone()
        red.enabled = False
        red([flat.params[0]])
        red.finish()
        ok_nosync = torch.equal(flat.grad, before)
        # broadcast of the flat parameters + floating buffers from rank 0
        m = _FakeModel(flat)
        broadcast_parameters(m)
        ok_bcast = torch.equal(flat.data, _FakeFlat(sizes, seed=100).data) and bool((m.running_mean == 0).all())
        gathered = all_gather_object({"rank": rank, "m_ap": 0.5 + rank})
        ok_gather = [g["rank"] for g in gathered] == list(range(world))
        q.put((rank, ok_sum, ok_nosync, ok_bcast and flat.refreshed, ok_gather))
    finally:
        dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_grad_allreduce_buckets_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, ok_sum, ok_nosync, ok_bcast, ok_gather in res:
        assert ok_sum, f"rank {rank}: bucketed all-reduce != sum of local grads"
        assert ok_nosync, f"rank {rank}: disabled reducer touched the gradient"
        assert ok_bcast, f"rank {rank}: broadcast_parameters"
        assert ok_gather, f"rank {rank}: all_gather_object"
