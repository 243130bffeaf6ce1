"""Isolated timing of the layer-1 bn3 GEMM pass (vcg_conv1x1_bn_res_relu), the statistics-only and storing conv3
GEMMs and the bn_apply pass it replaces, at the train step's shape (run from video-chapter-generation_amd/)."""
import torch, time
from vcg_hip import _lib, ops
_lib.call("vcg_init", 0)
D = "cuda"
M, N, K = 3211264, 256, 64
a2 = torch.relu(torch.randn(M, K, device=D)).to(torch.bfloat16)
x = torch.relu(torch.randn(M, N, device=D)).to(torch.bfloat16)
w = torch.randn(N, K, device=D) / 8
wf = ops.weight_fold(w, torch.ones(N, device=D), torch.bfloat16)
sh = torch.zeros(N, device=D)
st = ops.stats_buffer(N, M, D)
def t(f, n=5):
    f(); torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n): f()
    e1.record(); torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1e3
print("bnres alone us", t(lambda: ops.conv1x1_bn_res_relu(a2, wf, sh, x, M, N, K)))
print("stats-only us", t(lambda: ops.conv1x1_stats(a2, wf, st, M, N, K)))
y = torch.empty(M, N, device=D, dtype=torch.bfloat16)
print("stats+store us", t(lambda: ops.conv_fwd(a2.view(16, 448, 448, K), wf, 16, 448, 448, K, N, 1, 1, 1, 0, stats=st, out=y.view(16, 448, 448, N))))
print("stats-only then bnres us", t(lambda: (ops.conv1x1_stats(a2, wf, st, M, N, K), ops.conv1x1_bn_res_relu(a2, wf, sh, x, M, N, K))))
print("bn_apply us", t(lambda: ops.bn_apply(y, sh + 1, sh, N, relu=True, res=x, bits=True)))
