"""The torch.library registration of the vcg ops (vcg_hip/torch_ops.py): schemas exist and the fake
(meta) implementations infer output shapes / dtypes without a GPU."""
import torch
from torch._subclasses.fake_tensor import FakeTensorMode


def test_vcg_ops_registered_with_fake_impls():
    from vcg_hip import torch_ops  # noqa: F401
    for name in ("tsm_shift", "cross_entropy", "cross_entropy_bwd", "window_frames_u8", "linear"):
        assert hasattr(torch.ops.vcg, name), name
    with FakeTensorMode():
        x = torch.empty(8, 64, 7, 7)
        assert torch.ops.vcg.tsm_shift(x, 4, 8, 0).shape == x.shape
        lg = torch.empty(4, 2)
        assert torch.ops.vcg.cross_entropy(lg, torch.zeros(4, dtype=torch.int64)).shape == ()
        fr = torch.empty(10, 32, 32, 3, dtype=torch.uint8)
        y = torch.ops.vcg.window_frames_u8(fr, torch.zeros(2, 4, dtype=torch.int64), True, 4)
        assert y.shape == (8, 32, 32, 4) and y.dtype == torch.bfloat16
        assert torch.ops.vcg.linear(torch.empty(5, 16), torch.empty(8, 16), None, 1).shape == (5, 8)


def test_temporal_shift_and_cross_entropy_route_through_the_ops():
    import inspect
    from ops import temporal_shift
    from vcg_hip import functions
    assert "torch.ops.vcg.tsm_shift" in inspect.getsource(temporal_shift.TemporalShift.shift)
    assert "torch.ops.vcg.cross_entropy" in inspect.getsource(functions.cross_entropy)
