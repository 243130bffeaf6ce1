"""world_size-2 gloo tests (CPU) of the data-parallel exchange in vcg_hip/ddp.py: bucketed
all-reduce of a flat gradient buffer as parameters are reported final in backward order (buckets
flushed while hooks are still arriving), the bf16 wire format, no_sync-style micro-steps, rank-0
parameter broadcast, the per-forward BN-buffer broadcast and the metric gather."""
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
        from vcg_hip.ddp import BufferBroadcaster, GradAllReducer, all_gather_object, broadcast_parameters
        sizes = [1000, 300, 70000, 5, 2048, 77777, 256, 1]
        flat = _FakeFlat(sizes, seed=100 + rank)
        local = flat.grad.clone()
        red = GradAllReducer(flat, bucket_bytes=64 * 1024, record=True)  # small buckets: many flushes
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
        # overlap: buckets went out while the backward was still reporting parameters (a flush precedes the last
        # hook), every flush before finish() except the final one, and the flushed ranges tile the buffer once
        kinds = [e[0] for e in red.log]
        last_hook = max(i for i, k in enumerate(kinds) if k == "hook")
        flushes = [e for e in red.log if e[0] == "flush"]
        ok_overlap = kinds.index("flush") < last_hook and sum(1 for i, k in enumerate(kinds)
                                                               if k == "flush" and i > last_hook) <= 1
        covered = sorted((lo, hi) for _, lo, hi in flushes)
        ok_overlap = ok_overlap and all(a[1] <= b[0] for a, b in zip(covered, covered[1:])) and len(flushes) >= 3
        # bf16 wire format: the sum of the bf16-rounded local gradients, back in the fp32 buffer
        flat2 = _FakeFlat(sizes, seed=100 + rank)
        red2 = GradAllReducer(flat2, bucket_bytes=64 * 1024, wire_dtype=torch.bfloat16)
        for g in [[flat2.params[i] for i in grp] for grp in ([7, 6], [5], [4, 3], [2], [1, 0])]:
            red2(g)
        red2.finish()
        tot16 = torch.zeros_like(local)
        for r in range(world):
            tot16 += _FakeFlat(sizes, seed=100 + r).grad.bfloat16().float()
        ok_wire = torch.allclose(flat2.grad, tot16.bfloat16().float(), rtol=1e-2, atol=1e-2) and \
            flat2.grad.dtype == torch.float32
        # parameters no hook reports (the window model's heads) are still reduced, by finish()
        flat3 = _FakeFlat(sizes, seed=100 + rank)
        red3 = GradAllReducer(flat3, bucket_bytes=64 * 1024)
        red3([flat3.params[5]])
        red3([flat3.params[2]])
        red3.finish()
        ok_wire = ok_wire and torch.allclose(flat3.grad, total, rtol=0, atol=1e-5)
        # BN-buffer sync before each forward (DDP broadcast_buffers): rank 1's drifted stats become rank 0's
        mb = torch.nn.Module()
        mb.register_buffer("running_mean", torch.full((3,), 10.0 + rank))
        mb.register_buffer("running_var", torch.full((5,), 20.0 + rank))
        mb.register_buffer("num_batches_tracked", torch.tensor(rank))
        bb = BufferBroadcaster(mb)
        mb.running_mean.add_(rank)  # updates through the module's (re-bound) buffer
        bb()
        ok_bufs = bool((mb.running_mean == 10.0).all()) and bool((mb.running_var == 20.0).all()) and \
            int(mb.num_batches_tracked) == rank
        # a buffer replaced after binding (reassignment / .to()) is re-bound and still synced; mixed float dtypes
        # sync as one flat buffer per dtype
        mb.running_var = torch.full((5,), 30.0 + rank)
        mb.register_buffer("half_stat", torch.full((4,), 1.0 + rank, dtype=torch.float64))
        bb()
        ok_bufs = ok_bufs and bool((mb.running_var == 30.0).all()) and bool((mb.half_stat == 1.0).all()) and \
            len(bb.flats) == 2
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
        q.put((rank, ok_sum, ok_nosync, ok_bcast and flat.refreshed, ok_gather, ok_overlap, ok_wire, ok_bufs))
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
    for rank, ok_sum, ok_nosync, ok_bcast, ok_gather, ok_overlap, ok_wire, ok_bufs in res:
        assert ok_overlap, f"rank {rank}: buckets were not issued during the backward"
        assert ok_wire, f"rank {rank}: bf16 wire all-reduce"
        assert ok_bufs, f"rank {rank}: BufferBroadcaster"
        assert ok_sum, f"rank {rank}: bucketed all-reduce != sum of local grads"
        assert ok_nosync, f"rank {rank}: disabled reducer touched the gradient"
        assert ok_bcast, f"rank {rank}: broadcast_parameters"
        assert ok_gather, f"rank {rank}: all_gather_object"
