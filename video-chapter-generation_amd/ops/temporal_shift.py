"""Temporal Shift Module (drop-in for reference ops/temporal_shift.py).

`TemporalShift.shift` keeps the reference's signature and semantics (ops/temporal_shift.py:33-51):
for x viewed as [n_batch, n_segment, c, h, w] with fold = c // fold_div,
    out[:, t, :fold]        = x[:, t+1, :fold]        (zero at t = T-1)
    out[:, t, fold:2*fold]  = x[:, t-1, fold:2*fold]  (zero at t = 0)
    out[:, t, 2*fold:]      = x[:, t, 2*fold:]
It runs as the `vcg::tsm_shift` torch.library op over the `vcg_tsm_shift` HIP kernel (bit-exact gather; the
backward is the adjoint shift, the same op with direction 1).
Inside the native ResNet trunk the shift is not materialised at all: it is fused into conv1's
input gather (see vcg_hip/trunk.py), which is why `make_temporal_shift` only tags the convs.
"""
import torch
import torch.nn as nn

from vcg_hip import torch_ops  # noqa: F401  (registers torch.ops.vcg.*)


class TemporalShift(nn.Module):
    def __init__(self, net, n_segment=3, n_div=8, inplace=False):
        super().__init__()
        self.net = net
        self.n_segment = n_segment
        self.fold_div = n_div
        self.inplace = inplace  # the in-place variant computes the same values (temporal_shift.py:54-81)

    def forward(self, x):
        x = self.shift(x, self.n_segment, fold_div=self.fold_div, inplace=self.inplace)
        return self.net(x)

    @staticmethod
    def shift(x, n_segment, fold_div=3, inplace=False):
        nt, c, h, w = x.size()
        if nt % n_segment != 0:
            raise RuntimeError(f"TemporalShift: {nt} frames is not a multiple of n_segment={n_segment}")
        if x.dtype not in (torch.float32, torch.bfloat16):
            raise TypeError("TemporalShift: float32 / bfloat16 tensors only")
        return torch.ops.vcg.tsm_shift(x, n_segment, fold_div, 0)  # torch.library op (vcg_hip/torch_ops.py)


class TemporalPool(nn.Module):
    """Reference TemporalPool (temporal_shift.py:84-101) is not on the TwoStream path (temporal_pool=False)."""

    def __init__(self, net, n_segment):
        super().__init__()
        raise NotImplementedError("TemporalPool is not used by the video-segment-point path")


def make_temporal_shift(net, n_segment, n_div=8, place="blockres", temporal_pool=False):
    """Insert TemporalShift in front of every bottleneck conv1 (reference temporal_shift.py:104-146)."""
    from vcg_hip.nn import ResNet50
    if temporal_pool:
        raise NotImplementedError("temporal_pool=True is not used by the video-segment-point path")
    n_segment_list = [n_segment] * 4
    assert n_segment_list[-1] > 0
    if not isinstance(net, ResNet50):
        raise NotImplementedError(place)
    if "blockres" not in place:
        raise NotImplementedError(f"place={place!r}: the native trunk implements the reference's 'blockres' placement")
    n_round = 1
    if len(list(net.layer3.children())) >= 23:
        n_round = 2

    def make_block_temporal(stage, this_segment):
        blocks = list(stage.children())
        for i, b in enumerate(blocks):
            if i % n_round == 0:
                blocks[i].conv1 = TemporalShift(b.conv1, n_segment=this_segment, n_div=n_div)
        return nn.Sequential(*blocks)

    net.layer1 = make_block_temporal(net.layer1, n_segment_list[0])
    net.layer2 = make_block_temporal(net.layer2, n_segment_list[1])
    net.layer3 = make_block_temporal(net.layer3, n_segment_list[2])
    net.layer4 = make_block_temporal(net.layer4, n_segment_list[3])
