"""The vcg torch.library ops on the GPU (vcg_hip/torch_ops.py): torch.library.opcheck (schema, fake
implementation, autograd registration against the real kernels) and numerics -- the TSM shift and its autograd
adjoint bit-exact against the reference shift (ops/temporal_shift.py:33-51), cross-entropy within 1e-6 of torch's,
the frame ingest bit-identical to the ops path, linear within bf16 / fp32 tolerance of fp64."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _init():
    from vcg_hip import _lib, torch_ops  # noqa: F401
    _lib.call("vcg_init", 0)


def _tsm_ref(x, T, fold):
    nt, c, h, w = x.shape
    x = x.view(nt // T, T, c, h, w)
    out = torch.zeros_like(x)
    out[:, :-1, :fold] = x[:, 1:, :fold]
    out[:, 1:, fold:2 * fold] = x[:, :-1, fold:2 * fold]
    out[:, :, 2 * fold:] = x[:, :, 2 * fold:]
    return out.view(nt, c, h, w)


def test_opcheck():
    x = torch.randn(8, 64, 5, 5, device=DEV, requires_grad=True)
    torch.library.opcheck(torch.ops.vcg.tsm_shift, (x, 4, 8, 0))
    lg = torch.randn(6, 2, device=DEV, requires_grad=True)
    lab = torch.randint(0, 2, (6,), device=DEV)
    torch.library.opcheck(torch.ops.vcg.cross_entropy, (lg, lab))


def test_tsm_shift_op_and_adjoint_bitexact():
    from ops.temporal_shift import TemporalShift
    x = torch.randn(16, 64, 7, 7, device=DEV, requires_grad=True)
    y = TemporalShift.shift(x, 4, fold_div=8)
    assert torch.equal(y, _tsm_ref(x.detach(), 4, 8))
    g = torch.randn_like(y)
    y.backward(g)
    xr = x.detach().clone().requires_grad_()
    _tsm_ref(xr, 4, 8).backward(g)
    assert torch.equal(x.grad, xr.grad)


def test_cross_entropy_op():
    from vcg_hip.functions import cross_entropy
    lg = torch.randn(64, 2, device=DEV, requires_grad=True)
    lab = torch.randint(0, 2, (64,), device=DEV)
    loss = cross_entropy(lg, lab)
    loss.backward()
    lr = lg.detach().clone().requires_grad_()
    ref = F.cross_entropy(lr, lab)
    ref.backward()
    assert abs(loss.item() - ref.item()) < 1e-6
    assert (lg.grad - lr.grad).abs().max().item() < 1e-6


def test_window_frames_u8_op_matches_ops_path():
    from vcg_hip import ops
    fr = torch.randint(0, 256, (20, 32, 32, 3), dtype=torch.uint8, device=DEV)
    idx = torch.randint(0, 20, (3, 4), dtype=torch.int64, device=DEV)
    for bf16, dt in ((True, torch.bfloat16), (False, torch.float32)):
        a = torch.ops.vcg.window_frames_u8(fr, idx, bf16, 4)
        b = ops.window_frames_u8(fr, idx, dt, cpad=4)
        assert torch.equal(a, b)


@pytest.mark.parametrize("dt,tol", [(torch.float32, 1e-5), (torch.bfloat16, 2e-2)])
def test_linear_op(dt, tol):
    x = torch.randn(100, 64, device=DEV).to(dt)
    w = (torch.randn(48, 64, device=DEV) * 0.1).to(dt)
    b = torch.randn(48, device=DEV)
    y = torch.ops.vcg.linear(x, w, b, 1)
    ref = (x.double() @ w.double().T + b.double()).clamp_min(0)
    assert (y.double() - ref).abs().max().item() <= tol * ref.abs().max().item()


@pytest.mark.parametrize("dt,act,tol", [(torch.float32, 0, 1e-5), (torch.float32, 1, 1e-5), (torch.bfloat16, 0, 3e-2)])
def test_linear_op_autograd(dt, act, tol):
    """vcg::linear's backward (dX = dY' W, dW = dY'^T X, db = colsum(dY') on the GEMM / column-sum kernels) against
    float64 autograd of x W^T + b (+ ReLU); opcheck of the registration."""
    gen = torch.Generator().manual_seed(5)
    x0 = torch.randn(100, 64, generator=gen).to(DEV).to(dt)
    w0 = (torch.randn(48, 64, generator=gen) * 0.1).to(DEV).to(dt)
    b0 = torch.randn(48, generator=gen).to(DEV)
    g = torch.randn(100, 48, generator=gen).to(DEV).to(dt)
    x, w, b = (t.clone().requires_grad_() for t in (x0, w0, b0))
    y = torch.ops.vcg.linear(x, w, b, act)
    y.backward(g)
    xr, wr, br = (t.detach().double().requires_grad_() for t in (x0, w0, b0))
    yr = xr @ wr.T + br
    if act == 1:
        yr = yr.clamp_min(0)
    yr.backward(g.double())
    for a, r in ((x.grad, xr.grad), (w.grad, wr.grad), (b.grad, br.grad)):
        assert a.dtype == (torch.float32 if r is br.grad else dt)
        assert (a.double() - r).abs().max().item() <= tol * (r.abs().max().item() + 1e-12)
    if dt == torch.float32:
        torch.library.opcheck(torch.ops.vcg.linear, (x0.clone().requires_grad_(), w0.clone().requires_grad_(),
                                                     b0.clone().requires_grad_(), act))
