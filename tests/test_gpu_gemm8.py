"""The 256-row ping-pong GEMM kernel (csrc/igemm8.hip) against the 128 x 128 engine (VCG_G8=0) on the same inputs:
outputs bit for bit (every output fragment accumulates the same MFMAs in the same k order), the BatchNorm statistics
of EPI_STATS (finalized mean / invstd) to float rounding. VCG_G8=1 forces the kernel on every eligible shape.
Covers dense GEMMs with bias + activation (BERT-shaped, ragged M / K), 3x3 / stride-1 and stride-2 convs with
statistics (ragged M, 128- and 256-column tiles), the TSM-fused 1x1 conv, and a full-size layer-3 conv."""
import pytest
import torch

from vcg_hip import _lib, ops

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _init():
    _lib.call("vcg_init", 0)


def _rand(shape, seed, scale=1.0):
    g = torch.Generator().manual_seed(seed)
    return (torch.randn(shape, generator=g) * scale).to(torch.bfloat16).to(DEV)


def _both(monkeypatch, fn):
    outs = []
    for flag in ("1", "0"):
        monkeypatch.setenv("VCG_G8", flag)
        outs.append(fn())
        torch.cuda.synchronize()
    return outs


@pytest.mark.parametrize("M,N,K,act", [(8192, 768, 3072, ops.ACT_NONE), (8192, 3072, 768, ops.ACT_GELU),
                                       (1000, 256, 320, ops.ACT_RELU), (777, 384, 1000, ops.ACT_TANH)])
def test_gemm8_dense_store(monkeypatch, M, N, K, act):
    A, B = _rand((M, K), 1, 0.5), _rand((N, K), 2, 0.05)
    bias = (torch.randn(N, generator=torch.Generator().manual_seed(3)) * 0.1).to(DEV)
    a, b = _both(monkeypatch, lambda: ops.gemm(A, B, M, N, K, K, K, bias=bias, act=act))
    assert torch.equal(a, b), f"max |diff| {(a.float() - b.float()).abs().max().item():.3e}"


# (N, H, W, C, Cout, k, stride, pad, tsm T)
CONVS = [(8, 14, 14, 256, 256, 3, 1, 1, 0),    # layer-3 3x3, 256-column tiles, M = 1568 (ragged 256-row tile)
         (8, 28, 28, 128, 128, 3, 1, 1, 0),    # layer-2 3x3, 128-column tiles
         (8, 14, 14, 512, 256, 3, 2, 1, 0),    # stride 2
         (16, 7, 7, 512, 512, 3, 1, 1, 0),     # layer-4 3x3
         (8, 14, 14, 1024, 256, 1, 1, 0, 4),   # TSM-fused 1x1 conv1
         (16, 7, 7, 512, 2048, 1, 1, 0, 0)]    # conv3 of layer 4


@pytest.mark.parametrize("case", CONVS)
def test_gemm8_conv_stats(monkeypatch, case):
    N, H, W, C, Co, k, s, p, T = case
    x = _rand((N, H, W, C), 11)
    w = _rand((Co, k, k, C), 12, 0.05)
    OH, OW = ops.conv_out_hw(H, W, k, k, s, p)
    M = N * OH * OW
    fold = C // 8 if T else 0

    def run():
        st = ops.stats_buffer(Co, M, DEV)
        y = ops.conv_fwd(x, w, N, H, W, C, Co, k, k, s, p, T, fold, stats=st)
        mean, inv, sc, sh = (torch.empty(Co, device=DEV) for _ in range(4))
        ops.bn_finalize(st, ops.stats_tiles(M), M, Co, torch.ones(Co, device=DEV), torch.zeros(Co, device=DEV), mean,
                        inv, sc, sh)
        return y, mean, inv

    (ya, ma, ia), (yb, mb, ib) = _both(monkeypatch, run)
    assert torch.equal(ya, yb), f"max |diff| {(ya.float() - yb.float()).abs().max().item():.3e}"
    yd = ya.double().reshape(-1, Co)
    assert (ma.double() - yd.mean(0)).abs().max().item() < 1e-4 * (yd.abs().max().item() + 1)
    assert ((ia - ib).abs() / ib).max().item() < 1e-4


def test_gemm8_layer3_full(monkeypatch):
    """The benchmarked layer-3 3x3 conv (64 windows x 16 frames at 14 x 14) through both kernels."""
    N, H, W, C = 1024, 14, 14, 256
    x = _rand((N, H, W, C), 21)
    w = _rand((C, 3, 3, C), 22, 0.03)
    M = N * H * W

    def run():
        st = ops.stats_buffer(C, M, DEV)
        return ops.conv_fwd(x, w, N, H, W, C, C, 3, 3, 1, 1, stats=st)

    a, b = _both(monkeypatch, run)
    assert torch.equal(a, b)
